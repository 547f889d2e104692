// fileplan.cc — CHECK_FILE classification, md-raid0 geometry, chunk planning.
//
// classify_file() answers the reference's file_is_supported_nvme()
// (kmod/nvme_strom.c:373-465) from userspace: fstatfs for the filesystem,
// /sys/dev/block/<maj:min> for the backing disk, /sys/block/mdX/md for
// raid0 geometry and members, and device/numa_node for locality.  Strict
// mode enforces the reference's acceptance rules (ext4/xfs on raw NVMe or
// md-raid0 of NVMe); the default also admits any filesystem that accepts
// O_DIRECT, because the userspace engine does not need to own the
// block-to-LBA translation.
//
// plan_chunks() is the semantic core of do_memcpy_ssd2gpu/ssd2ram
// (:1488-1604, :1767-1884) and memcpy_from_nvme_ssd (:1303-1405):
// relseg modulo addressing, the page-cache majority score, SSD chunks
// packed from the head with RAM chunks from the tail (SSD2GPU), the
// merge rule (contiguous source, contiguous destination, <= max request,
// no destination segment crossing, no raid0 chunk crossing).  It also
// fixes reference defect #10: a chunk that starts at or past EOF is
// rejected with -ERANGE.
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/statfs.h>
#include <sys/sysmacros.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <set>

#include "engine.h"

namespace strom {

static bool read_text(const std::string &path, std::string *out) {
  std::ifstream f(path);
  if (!f) return false;
  std::string s((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  *out = s;
  return true;
}

static long read_long(const std::string &path, long dflt) {
  std::string s;
  if (!read_text(path, &s) || s.empty()) return dflt;
  return strtol(s.c_str(), nullptr, 0);
}

static bool is_nvme_ns_name(const std::string &n) {
  // nvme<ctrl>n<ns> (optionally a partition suffix p<k> is stripped earlier)
  unsigned a, b;
  char tail;
  return sscanf(n.c_str(), "nvme%un%u%c", &a, &b, &tail) == 2;
}

static int disk_numa_node(const std::string &disk) {
  const char *cands[] = {"/device/numa_node", "/device/device/numa_node"};
  for (const char *c : cands) {
    long v = read_long("/sys/block/" + disk + c, LONG_MIN);
    if (v != LONG_MIN) return (int)v;
  }
  return -1;
}

static const char *fs_name_of(uint64_t magic) {
  switch (magic) {
    case 0xEF53: return "ext4";
    case 0x58465342: return "xfs";
    case 0x794c7630: return "overlay";
    case 0x01021994: return "tmpfs";
    case 0x9123683E: return "btrfs";
    case 0x2FC12FC1: return "zfs";
    case 0x6969: return "nfs";
    default: return "other";
  }
}

// Build raid0 zones from sysfs: members sorted by size give the zones
// (drivers/md/raid0.c create_strip_zones semantics, re-derived), in the
// shared core's geometry struct.
static int load_raid0(const std::string &md, FileClass *fc) {
  std::string base = "/sys/block/" + md + "/md/";
  std::string level;
  if (!read_text(base + "level", &level) || level != "raid0") return -ENOTSUP;
  long layout = read_long(base + "layout", 0);
  if (layout != 0 && layout != 1 && layout != 2) return -ENOTSUP;
  long chunk_bytes = read_long(base + "chunk_size", 0);
  if (chunk_bytes < 4096 || (chunk_bytes % 4096)) return -ENOTSUP;
  Raid0Geometry &g = fc->raid0;
  memset(&g, 0, sizeof g);
  g.chunk_sects = (uint32_t)(chunk_bytes >> 9);
  struct Mem { std::string name; uint64_t sectors; uint64_t off; int slot; };
  std::vector<Mem> mem;
  DIR *d = opendir(base.c_str());
  if (!d) return -ENOTSUP;
  while (dirent *e = readdir(d)) {
    if (strncmp(e->d_name, "dev-", 4) != 0) continue;
    std::string dd = base + e->d_name + "/";
    char link[PATH_MAX];
    ssize_t n = readlink((dd + "block").c_str(), link, sizeof link - 1);
    if (n <= 0) continue;
    link[n] = 0;
    Mem m;
    m.name = strrchr(link, '/') ? strrchr(link, '/') + 1 : link;
    m.slot = (int)read_long(dd + "slot", (long)mem.size());
    m.off = (uint64_t)read_long(dd + "offset", 0);
    m.sectors = (uint64_t)read_long(dd + "size", 0) * 2;  // KiB -> sectors
    mem.push_back(m);
  }
  closedir(d);
  if (mem.empty() || mem.size() > STROM_RAID0_MAX_DISKS) return -ENOTSUP;
  std::sort(mem.begin(), mem.end(), [](const Mem &a, const Mem &b) { return a.slot < b.slot; });
  g.ndisks = (uint32_t)mem.size();
  for (size_t i = 0; i < mem.size(); ++i) {
    fc->members.push_back(mem[i].name);
    g.data_offset[i] = mem[i].off;
  }
  std::set<uint64_t> sizes;
  for (auto &m : mem) sizes.insert(m.sectors / g.chunk_sects * g.chunk_sects);
  uint64_t prev = 0, md_end = 0;
  for (uint64_t sz : sizes) {
    if (sz == prev) continue;
    if (g.nzones == STROM_RAID0_MAX_ZONES) return -ENOTSUP;
    const uint32_t z = g.nzones++;
    for (size_t i = 0; i < mem.size(); ++i)
      if (mem[i].sectors / g.chunk_sects * g.chunk_sects >= sz)
        g.zone_devs[z][g.zone_nb_dev[z]++] = (uint8_t)i;
    md_end += (sz - prev) * g.zone_nb_dev[z];
    g.zone_end[z] = md_end;
    g.zone_dev_start[z] = prev;
    prev = sz;
  }
  return strom_core_raid0_check(&g) ? -ENOTSUP : 0;
}

int classify_file(int fd, FileClass *fc, bool strict) {
  struct stat st;
  if (fstat(fd, &st) != 0) return -errno;
  int fl = fcntl(fd, F_GETFL);
  if (fl < 0) return -errno;
  if ((fl & O_ACCMODE) == O_WRONLY) return -EBADF;
  // directories are accepted too: PostgreSQL probes a tablespace's
  // database directory (reference pgsql/nvme_strom.c:192-280)
  const bool is_dir = S_ISDIR(st.st_mode);
  if (!S_ISREG(st.st_mode) && !is_dir) return -ENOTSUP;
  struct statfs sf;
  if (fstatfs(fd, &sf) != 0) return -errno;
  fc->dev = st.st_dev;
  fc->ino = st.st_ino;
  fc->size = st.st_size;
  fc->fs_bsize = (uint32_t)sf.f_bsize;
  fc->fs_magic = (uint64_t)sf.f_type;
  fc->fs_name = fs_name_of(fc->fs_magic);
  if (!is_dir && st.st_size < 4096) return -ENOTSUP;  // i_size >= PAGE_SIZE
  if (sf.f_bsize > 4096 && (fc->fs_name == "ext4" || fc->fs_name == "xfs"))
    return -ENOTSUP;                                   // blocksize <= PAGE_SIZE

  // backing block device
  char sys[128];
  snprintf(sys, sizeof sys, "/sys/dev/block/%u:%u", major(st.st_dev), minor(st.st_dev));
  char real[PATH_MAX];
  if (major(st.st_dev) != 0 && realpath(sys, real)) {
    std::string p = real;
    std::string name = p.substr(p.rfind('/') + 1);
    std::string disk = name;
    if (access((p + "/partition").c_str(), F_OK) == 0) {
      fc->part_start_sect = (uint64_t)read_long(p + "/start", 0);
      std::string parent = p.substr(0, p.rfind('/'));
      disk = parent.substr(parent.rfind('/') + 1);
    }
    fc->disk = disk;
    if (is_nvme_ns_name(disk)) {
      fc->nvme = true;
      fc->numa_node = disk_numa_node(disk);
    } else if (disk.compare(0, 2, "md") == 0 && load_raid0(disk, fc) == 0) {
      bool all_nvme = !fc->members.empty();
      std::set<int> nodes;
      for (auto &m : fc->members) {
        std::string mdisk = m;
        // members may be partitions: strip pN
        size_t pp = mdisk.rfind('p');
        if (!is_nvme_ns_name(mdisk) && pp != std::string::npos && is_nvme_ns_name(mdisk.substr(0, pp)))
          mdisk = mdisk.substr(0, pp);
        if (!is_nvme_ns_name(mdisk)) all_nvme = false;
        nodes.insert(disk_numa_node(mdisk));
      }
      fc->md_raid0 = all_nvme || !strict;
      fc->numa_node = nodes.size() == 1 ? *nodes.begin() : -1;
      if (strict && !all_nvme) return -ENOTSUP;
    }
  }
  if (strict) {
    if (fc->fs_name != "ext4" && fc->fs_name != "xfs") return -ENOTSUP;
    if (!fc->nvme && !fc->md_raid0) return -ENOTSUP;
  }
  fc->dma64 = true;  // staging/destination pages are ours: any address
  return 0;
}

// PCI function (domain:bus:dev.fn) of the NVMe controller behind a
// namespace disk: /sys/block/<disk>/device resolves to .../<bdf>/nvme/nvmeX
// for a plain controller; a multipath head resolves to its nvme-subsystem,
// whose first controller link is used.
static bool is_bdf(const std::string &c) {
  unsigned d, b, v, f;
  char tail;
  return c.size() == 12 && sscanf(c.c_str(), "%4x:%2x:%2x.%1x%c", &d, &b, &v, &f, &tail) == 4;
}

static std::string bdf_in_path(const std::string &p) {
  std::string last;
  size_t i = 0;
  while (i < p.size()) {
    size_t j = p.find('/', i);
    if (j == std::string::npos) j = p.size();
    std::string c = p.substr(i, j - i);
    if (is_bdf(c)) last = c;
    i = j + 1;
  }
  return last;
}

std::string nvme_controller_bdf(const std::string &disk) {
  char real[PATH_MAX];
  std::string dev = "/sys/block/" + disk + "/device";
  if (!realpath(dev.c_str(), real)) return "";
  std::string p = real;
  if (p.find("nvme-subsystem") != std::string::npos) {
    if (DIR *d = opendir(p.c_str())) {
      std::string found;
      while (struct dirent *e = readdir(d)) {
        unsigned c;
        char tail;
        if (sscanf(e->d_name, "nvme%u%c", &c, &tail) != 1) continue;
        std::string q = p + "/" + e->d_name;
        if (realpath(q.c_str(), real)) found = bdf_in_path(real);
        if (!found.empty()) break;
      }
      closedir(d);
      return found;
    }
    return "";
  }
  return bdf_in_path(p);
}

// ------------------------------------------------------------- planning
namespace {
int plan_submit(void *ctx, const strom_extent *e) {
  auto *out = (ChunkPlan *)ctx;
  out->ssd.push_back(IoRange{e->file_off, e->dest, e->len, e->member, e->sect});
  return 0;
}
int ident_bmap(void *, uint64_t fblk, uint64_t *dblk) {
  *dblk = fblk;
  return 0;
}
}  // namespace

// Placement, residency routing and merging come from the shared core
// (kmod/strom_core.c): the kernel provider plans with the same code.
int plan_chunks(const PlanParams &p, ChunkPlan *out) {
  const uint32_t cs = p.chunk_sz;
  if (cs < 4096 || (cs & 4095) || cs > std::max(p.max_request, STROM_LEGACY_MAX_REQUEST))
    return -EINVAL;
  out->ids_out.assign(p.nr_chunks, 0);
  out->ssd.clear();
  out->ram_fpos.clear();
  out->ram_dest.clear();
  out->nr_ram = out->nr_ssd = out->nr_submit = out->nr_blocks = 0;
  const uint32_t threshold = strom_core_cache_threshold(cs >> 12);

  strom_landing land{p.nr_chunks, 0, 0, p.reorder};
  strom_planner pl;
  memset(&pl, 0, sizeof pl);
  pl.max_req = std::max<uint32_t>(p.max_request, cs);
  pl.file_contig = true;      // reads go by file offset
  pl.dest_segment = p.dest_segment;
  pl.blkbits = 12;
  // raid0 splits need volume sectors: only with a real block map
  pl.raid0 = p.bmap ? p.raid0 : nullptr;
  pl.part_start_sect = p.bmap ? p.part_start_sect : 0;
  pl.bmap = p.bmap ? p.bmap : ident_bmap;
  pl.bmap_ctx = p.bmap_ctx;
  pl.submit = plan_submit;
  pl.submit_ctx = out;
  strom_core_planner_init(&pl);

  for (uint32_t i = 0; i < p.nr_chunks; ++i) {
    const uint32_t cid = p.ids[i];
    uint64_t fpos = 0;
    if (strom_core_chunk_fpos(cid, cs, p.relseg_sz, p.file_size, &fpos)) return -ERANGE;
    bool cached = false;
    if (p.resident) {
      // mincore cannot see dirty pages; O_DIRECT writes them back first
      const long r = p.resident(fpos, cs);
      cached = r > 0 && strom_core_cache_wins((uint32_t)r, threshold);
    }
    const uint32_t slot = strom_core_land(&land, i, cached);
    out->ids_out[slot] = cid;
    const uint64_t dest = (uint64_t)slot * cs;
    if (cached) {
      out->ram_fpos.push_back(fpos);
      out->ram_dest.push_back(dest);
      continue;
    }
    int rc = strom_core_plan_range(&pl, fpos, cs, dest);
    if (rc) return rc;
  }
  int rc = strom_core_plan_flush(&pl);
  if (rc) return rc;
  out->nr_ram = land.nr_ram;
  out->nr_ssd = land.nr_ssd;
  out->nr_submit = pl.nr_submit;
  out->nr_blocks = (uint32_t)pl.nr_sectors;
  return 0;
}

// Exact extent reads (MEMCPY_SSD2GPU_EXTENTS): the shared core lays the
// extents out in runs and feeds them to the same merge rules; no residency
// routing (every byte from storage, O_DIRECT being coherent with dirty
// pages).  planner == false: layout only.
int plan_xfer(const PlanParams &p, strom_file_extent *x, uint32_t n, uint32_t gap_max,
              bool planner, ChunkPlan *out, uint64_t *dst_bytes, uint64_t *read_bytes) {
  static_assert(sizeof(strom_file_extent) == sizeof(strom_xfer_extent), "extent layout");
  static_assert(offsetof(strom_file_extent, dst_off) == offsetof(strom_xfer_extent, dst_off) &&
                offsetof(strom_file_extent, len) == offsetof(strom_xfer_extent, len), "extent layout");
  out->ssd.clear();
  out->ram_fpos.clear();
  out->ram_dest.clear();
  out->ids_out.clear();
  out->nr_ram = out->nr_ssd = out->nr_submit = out->nr_blocks = 0;
  strom_planner pl;
  memset(&pl, 0, sizeof pl);
  pl.max_req = std::max<uint32_t>(p.max_request, 4096);
  pl.file_contig = true;
  pl.blkbits = 12;
  pl.raid0 = p.bmap ? p.raid0 : nullptr;
  pl.part_start_sect = p.bmap ? p.part_start_sect : 0;
  pl.bmap = p.bmap ? p.bmap : ident_bmap;
  pl.bmap_ctx = p.bmap_ctx;
  pl.submit = plan_submit;
  pl.submit_ctx = out;
  strom_core_planner_init(&pl);
  int rc = strom_core_plan_xfer(planner ? &pl : nullptr, (strom_xfer_extent *)x, n, gap_max,
                                p.file_size, dst_bytes, read_bytes);
  if (!rc && planner) rc = strom_core_plan_flush(&pl);
  if (rc) return rc;
  out->nr_submit = pl.nr_submit;
  out->nr_blocks = (uint32_t)pl.nr_sectors;
  out->nr_ssd = (uint32_t)out->ssd.size();
  return 0;
}

}  // namespace strom

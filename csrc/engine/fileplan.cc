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
// (drivers/md/raid0.c create_strip_zones semantics, re-derived).
static int load_raid0(const std::string &md, FileClass *fc) {
  std::string base = "/sys/block/" + md + "/md/";
  std::string level;
  if (!read_text(base + "level", &level) || level != "raid0") return -ENOTSUP;
  long layout = read_long(base + "layout", 0);
  if (layout != 0 && layout != 1 && layout != 2) return -ENOTSUP;
  long chunk_bytes = read_long(base + "chunk_size", 0);
  if (chunk_bytes < 4096 || (chunk_bytes % 4096)) return -ENOTSUP;
  fc->raid0.chunk_sects = (uint32_t)(chunk_bytes >> 9);
  struct Mem { std::string name; uint64_t sectors; uint64_t off; int slot; };
  std::vector<Mem> mem;
  DIR *d = opendir(base.c_str());
  if (!d) return -ENOTSUP;
  while (dirent *e = readdir(d)) {
    if (strncmp(e->d_name, "dev-", 4) != 0) continue;
    std::string dd = base + e->d_name + "/";
    std::string blk;
    char link[PATH_MAX];
    ssize_t n = readlink((dd + "block").c_str(), link, sizeof link - 1);
    if (n <= 0) continue;
    link[n] = 0;
    blk = strrchr(link, '/') ? strrchr(link, '/') + 1 : link;
    Mem m;
    m.name = blk;
    m.slot = (int)read_long(dd + "slot", (long)mem.size());
    m.off = (uint64_t)read_long(dd + "offset", 0);
    m.sectors = (uint64_t)read_long(dd + "size", 0) * 2;  // KiB -> sectors
    mem.push_back(m);
  }
  closedir(d);
  if (mem.empty()) return -ENOTSUP;
  std::sort(mem.begin(), mem.end(), [](const Mem &a, const Mem &b) { return a.slot < b.slot; });
  fc->raid0.data_offset.clear();
  for (auto &m : mem) {
    fc->members.push_back(m.name);
    fc->raid0.data_offset.push_back(m.off);
  }
  // zones: distinct member sizes rounded to the chunk
  std::set<uint64_t> sizes;
  for (auto &m : mem) sizes.insert(m.sectors / fc->raid0.chunk_sects * fc->raid0.chunk_sects);
  uint64_t prev = 0, md_end = 0;
  for (uint64_t sz : sizes) {
    std::vector<int> devs;
    for (size_t i = 0; i < mem.size(); ++i)
      if (mem[i].sectors / fc->raid0.chunk_sects * fc->raid0.chunk_sects >= sz) devs.push_back((int)i);
    if (sz == prev) continue;
    md_end += (sz - prev) * devs.size();
    fc->raid0.zone_end.push_back(md_end);
    fc->raid0.zone_dev_start.push_back(prev);
    fc->raid0.zone_devs.push_back(devs);
    prev = sz;
  }
  return 0;
}

int Raid0Geometry::map(uint64_t sector, uint32_t nr, int *member, uint64_t *msector) const {
  if (chunk_sects == 0 || zone_end.empty()) return -EINVAL;
  size_t z = 0;
  while (z < zone_end.size() && sector >= zone_end[z]) ++z;
  if (z == zone_end.size()) return -ERANGE;
  uint64_t zstart = z ? zone_end[z - 1] : 0;
  uint64_t in_chunk = sector % chunk_sects;
  if (in_chunk + nr > chunk_sects) return -ESPIPE;  // request straddles a stripe
  const std::vector<int> &devs = zone_devs[z];
  uint64_t off = sector - zstart;
  uint64_t chunk_no = off / chunk_sects;             // chunk index inside the zone
  uint64_t row = chunk_no / devs.size();
  int dev = devs[chunk_no % devs.size()];
  *member = dev;
  *msector = zone_dev_start[z] + row * chunk_sects + in_chunk + data_offset[dev];
  return 0;
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

// ------------------------------------------------------------- planning
int plan_chunks(const PlanParams &p, ChunkPlan *out) {
  const uint32_t cs = p.chunk_sz;
  if (cs < 4096 || (cs & 4095) || cs > std::max(p.max_request, STROM_LEGACY_MAX_REQUEST))
    return -EINVAL;
  out->ids_out.assign(p.nr_chunks, 0);
  out->ssd.clear();
  out->ram_fpos.clear();
  out->ram_dest.clear();
  out->nr_ram = out->nr_ssd = out->nr_submit = out->nr_blocks = 0;
  const uint32_t npages = cs >> 12;
  const long threshold = npages / 2;
  const uint32_t max_req = std::max<uint32_t>(p.max_request, cs);

  IoRange cur{0, 0, 0, -1};
  auto flush = [&]() {
    if (cur.len) {
      out->ssd.push_back(cur);
      out->nr_submit++;
      out->nr_blocks += cur.len >> 9;
      cur.len = 0;
    }
  };
  uint64_t ssd_dest = 0;
  for (uint32_t i = 0; i < p.nr_chunks; ++i) {
    uint64_t cid = p.ids[i];
    uint64_t fpos = (p.relseg_sz ? cid % p.relseg_sz : cid) * (uint64_t)cs;
    if (fpos >= p.file_size) return -ERANGE;
    long score = 0;
    if (p.resident) {
      long r = p.resident(fpos, cs);
      if (r > 0) score = r;
    }
    if (score > threshold) {
      uint64_t dest;
      if (p.reorder) {
        out->nr_ram++;
        uint32_t pos = p.nr_chunks - out->nr_ram;
        out->ids_out[pos] = (uint32_t)cid;
        dest = (uint64_t)pos * cs;
      } else {
        out->nr_ram++;
        out->ids_out[i] = (uint32_t)cid;
        dest = (uint64_t)i * cs;
      }
      out->ram_fpos.push_back(fpos);
      out->ram_dest.push_back(dest);
      continue;
    }
    uint64_t dest = p.reorder ? ssd_dest : (uint64_t)i * cs;
    if (p.reorder) {
      out->ids_out[out->nr_ssd] = (uint32_t)cid;
      ssd_dest += cs;
    } else {
      out->ids_out[i] = (uint32_t)cid;
    }
    out->nr_ssd++;
    // walk the chunk in 4 KiB pages (raid0 may split it), merging as we go
    for (uint32_t pg = 0; pg < npages;) {
      uint64_t f = fpos + (uint64_t)pg * 4096;
      uint64_t d = dest + (uint64_t)pg * 4096;
      uint32_t run = npages - pg;  // pages we may take in one piece
      int member = -1;
      if (p.raid0) {
        // pages to the end of the current stripe chunk
        uint64_t sect = (f >> 9) + p.part_start_sect;
        uint64_t in_chunk = sect % p.raid0->chunk_sects;
        uint32_t left = (uint32_t)((p.raid0->chunk_sects - in_chunk) >> 3);
        if (left == 0) left = 1;
        run = std::min(run, left);
        uint64_t msect;
        int rc = p.raid0->map(sect, run * 8, &member, &msect);
        if (rc) return rc;
      }
      uint32_t bytes = run * 4096;
      bool seg_ok = true;
      if (p.dest_segment) {
        // the merged request may not cross a destination segment
        seg_ok = (cur.dest_off / p.dest_segment) == ((d + bytes - 1) / p.dest_segment);
      }
      if (cur.len && cur.member == member && cur.file_off + cur.len == f &&
          cur.dest_off + cur.len == d && seg_ok && cur.len + bytes <= max_req) {
        cur.len += bytes;
      } else if (cur.len && cur.member == member && cur.file_off + cur.len == f &&
                 cur.dest_off + cur.len == d && seg_ok && cur.len < max_req) {
        // fill the current request up to max_req, continue with the rest
        uint32_t take = max_req - cur.len;
        cur.len += take;
        flush();
        pg += take / 4096;
        continue;
      } else {
        flush();
        if (p.dest_segment) {
          // never start a request that crosses a segment: trim the run
          uint64_t seg_end = (d / p.dest_segment + 1) * p.dest_segment;
          if (d + bytes > seg_end) bytes = (uint32_t)(seg_end - d);
        }
        if (bytes > max_req) bytes = max_req;
        cur = IoRange{f, d, bytes, member};
      }
      pg += bytes / 4096;
    }
  }
  flush();
  return 0;
}

}  // namespace strom

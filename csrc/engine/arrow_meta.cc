// arrow_meta.cc — record-batch headers of an Arrow IPC file, read and
// parsed natively.
//
// An Arrow IPC file keeps one flatbuffer Message per record batch in front
// of each body; the footer lists where they are (File.fbs Block: offset,
// metaDataLength, bodyLength).  Opening a file for a GPU scan needs every
// header (buffer offsets and lengths, row counts, body compression), i.e.
// thousands of small reads spread over the file — on a cold file one
// storage round trip each.  strom_arrow_headers() issues them from a few
// threads at once and decodes the Message -> RecordBatch tables
// (Message.fbs: Message{version, header_type, header, bodyLength},
// RecordBatch{length, nodes:[FieldNode], buffers:[Buffer], compression},
// BodyCompression{codec, method}) with bounds-checked flatbuffer reads: the
// file is input data, so a malformed header is an error, never an
// out-of-range access.  nvme_strom_amd/utils/arrow_ipc.py holds the same
// walk in Python (tests pin the two against each other and against
// pyarrow's own files).
#include <errno.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

namespace {

struct Fb {
  const uint8_t *b;
  uint64_t n;

  template <class T>
  bool get(uint64_t off, T *v) const {
    if (off > n || n - off < sizeof(T)) return false;
    memcpy(v, b + off, sizeof(T));
    return true;
  }
};

// table at `pos`: its vtable and field lookups
struct Table {
  const Fb *f;
  uint64_t pos = 0, vt = 0;
  uint16_t vtlen = 0;

  bool open(const Fb *fb, uint64_t p) {
    f = fb;
    pos = p;
    int32_t d;
    if (!f->get(p, &d)) return false;
    const int64_t v = (int64_t)p - d;
    if (v < 0) return false;
    vt = (uint64_t)v;
    return f->get(vt, &vtlen) && vtlen >= 4;
  }
  // field offset inside the table (0: absent)
  bool field(int i, uint16_t *fo) const {
    const uint64_t o = 4 + 2 * (uint64_t)i;
    if (o + 2 > vtlen) {
      *fo = 0;
      return true;
    }
    return f->get(vt + o, fo);
  }
  template <class T>
  bool scalar(int i, T *v, T dflt) const {
    uint16_t fo;
    if (!field(i, &fo)) return false;
    if (!fo) {
      *v = dflt;
      return true;
    }
    return f->get(pos + fo, v);
  }
  // referenced object position (table or vector); *present false if absent
  bool ref(int i, uint64_t *p, bool *present) const {
    uint16_t fo;
    if (!field(i, &fo)) return false;
    *present = fo != 0;
    if (!fo) return true;
    uint32_t u;
    if (!f->get(pos + fo, &u)) return false;
    *p = pos + fo + u;
    return *p < f->n;
  }
  bool table(int i, Table *t, bool *present) const {
    uint64_t p;
    if (!ref(i, &p, present)) return false;
    return !*present || t->open(f, p);
  }
  // vector of `esz`-byte structs: element start and count, fully in bounds
  bool vector(int i, uint64_t esz, uint64_t *start, uint32_t *cnt) const {
    uint64_t p;
    bool present;
    if (!ref(i, &p, &present)) return false;
    if (!present) {
      *start = 0;
      *cnt = 0;
      return true;
    }
    if (!f->get(p, cnt)) return false;
    *start = p + 4;
    return *start <= f->n && (f->n - *start) / esz >= *cnt;
  }
};

enum : int32_t { kNotBatch = -2, kNoCodec = -1 };

// one header; false: malformed
bool parse_one(const uint8_t *buf, uint64_t len, int32_t max_nodes, int32_t max_bufs, int64_t *rows,
               int32_t *codec, int32_t *nn, int32_t *nb, int64_t *nodes, int64_t *bufs) {
  Fb fb{buf, len};
  int32_t cont;
  if (!fb.get(0, &cont)) return false;
  uint64_t root = cont == -1 ? 8 : 4;   // continuation marker, or the legacy length prefix
  uint32_t u;
  if (!fb.get(root, &u)) return false;
  Table msg;
  if (!msg.open(&fb, root + u)) return false;
  uint8_t htype;
  if (!msg.scalar(1, &htype, (uint8_t)0)) return false;
  if (htype != 3) {                     // not a RecordBatch (dictionary batch, ...)
    *codec = kNotBatch;
    *nn = *nb = 0;
    *rows = 0;
    return true;
  }
  Table rb;
  bool present;
  if (!msg.table(2, &rb, &present) || !present) return false;
  if (!rb.scalar(0, rows, (int64_t)0)) return false;
  Table comp;
  if (!rb.table(3, &comp, &present)) return false;
  *codec = kNoCodec;
  if (present) {
    int8_t c;
    if (!comp.scalar(0, &c, (int8_t)0)) return false;
    *codec = c;
  }
  uint64_t s;
  uint32_t cnt;
  if (!rb.vector(1, 16, &s, &cnt) || cnt > (uint32_t)max_nodes) return false;
  *nn = (int32_t)cnt;
  memcpy(nodes, buf + s, 16 * (uint64_t)cnt);
  if (!rb.vector(2, 16, &s, &cnt) || cnt > (uint32_t)max_bufs) return false;
  *nb = (int32_t)cnt;
  memcpy(bufs, buf + s, 16 * (uint64_t)cnt);
  return true;
}

}  // namespace

// blocks: n x {offset, metaDataLength, bodyLength} (the footer's Block
// structs).  Outputs per block k: rows[k], codec[k] (-1 none, 0 LZ4_FRAME,
// 1 ZSTD, -2 not a record batch), nnodes[k] / nbufs[k] and the FieldNode /
// Buffer structs (2 x int64 each) at nodes[k * max_nodes * 2] /
// bufs[k * max_bufs * 2].  Returns 0, -errno of a failed read, or
// -EBADMSG with *bad = the first malformed block.
extern "C" int strom_arrow_headers(int fd, const int64_t *blocks, int64_t n, int32_t max_nodes,
                                   int32_t max_bufs, int64_t *rows, int32_t *codec,
                                   int32_t *nnodes, int32_t *nbufs, int64_t *nodes, int64_t *bufs,
                                   int32_t threads, int64_t *bad) {
  if (n < 0 || max_nodes < 0 || max_bufs < 0 || !bad) return -EINVAL;
  *bad = -1;
  std::atomic<int64_t> next{0};
  std::atomic<int> err{0};
  std::atomic<int64_t> first_bad{INT64_MAX};
  auto work = [&] {
    std::vector<uint8_t> buf;
    for (;;) {
      const int64_t k = next.fetch_add(1);
      if (k >= n || err.load(std::memory_order_relaxed)) return;
      const int64_t off = blocks[3 * k], len = blocks[3 * k + 1];
      if (off < 0 || len < 8 || len > (64 << 20)) {
        int64_t cur = first_bad.load();
        while (k < cur && !first_bad.compare_exchange_weak(cur, k)) {
        }
        continue;
      }
      buf.resize((size_t)len);
      int64_t got = 0;
      while (got < len) {
        const ssize_t r = pread(fd, buf.data() + got, (size_t)(len - got), off + got);
        if (r < 0) {
          if (errno == EINTR) continue;
          err.store(-errno);
          return;
        }
        if (r == 0) break;
        got += r;
      }
      if (got < len || !parse_one(buf.data(), (uint64_t)len, max_nodes, max_bufs, &rows[k],
                                  &codec[k], &nnodes[k], &nbufs[k],
                                  nodes + 2 * (uint64_t)max_nodes * k,
                                  bufs + 2 * (uint64_t)max_bufs * k)) {
        int64_t cur = first_bad.load();
        while (k < cur && !first_bad.compare_exchange_weak(cur, k)) {
        }
      }
    }
  };
  const int nt = threads < 1 ? 1 : threads > 64 ? 64 : threads;
  std::vector<std::thread> pool;
  for (int i = 1; i < nt && i < n; ++i) pool.emplace_back(work);
  work();
  for (auto &t : pool) t.join();
  if (err.load()) return err.load();
  if (first_bad.load() != INT64_MAX) {
    *bad = first_bad.load();
    return -EBADMSG;
  }
  return 0;
}

// Mutation test of the zstd decoder's phases (csrc/kernels/zstd.hip, host
// copies: strom_zstd_host, strom_zstd_host_fp — the frame-parallel
// decoder, 4 waves per stream — and strom_zstd_host_lp, the lane-parallel
// one, whose literals decode into the output buffer's tail), built host-only with ASan + UBSan
// (make build/zstd_fuzz): every seed frame must decode to its reference
// output, and random edits / truncations of it (byte flips, bit flips,
// a cut tail) must end in a clean status, never an out-of-range access —
// the GPU kernel runs the same bounds checks.
//
//   zstd_fuzz ITERATIONS SEED.zst SEED.raw [SEED.zst SEED.raw ...]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

extern "C" int strom_zstd_host(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst,
                               uint32_t cap);
extern "C" int strom_zstd_host_fp(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst,
                                  uint32_t cap, uint32_t nw);
struct Desc {
  uint64_t src_off, dst_off;
  uint32_t src_len, dst_len;
};
extern "C" int strom_zstd_host_lp(int codec, const uint8_t *src, const Desc *desc, uint32_t n,
                                  uint8_t *dst, int32_t *status, double ent_factor);

// one stream through the lane-parallel phases
static int lp1(const uint8_t *src, uint32_t len, uint8_t *dst, uint32_t cap) {
  const Desc d{0, 0, len, cap};
  int32_t st = 0;
  if (strom_zstd_host_lp(7, src, &d, 1, dst, &st, 0) < 0) return -999;
  return st;
}

static std::vector<uint8_t> slurp(const char *path) {
  std::vector<uint8_t> v;
  FILE *f = fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(f);
  return v;
}

int main(int argc, char **argv) {
  if (argc < 4 || (argc - 2) % 2) {
    fprintf(stderr, "usage: %s ITERS SEED.zst SEED.raw ...\n", argv[0]);
    return 2;
  }
  const int iters = atoi(argv[1]);
  std::mt19937_64 rng(1234);
  long ok = 0, rejected = 0, decoded = 0;
  for (int a = 2; a < argc; a += 2) {
    const std::vector<uint8_t> z = slurp(argv[a]), raw = slurp(argv[a + 1]);
    if (z.empty()) return 2;
    const uint32_t cap = (uint32_t)raw.size();
    // exact-size heap buffers: ASan sees any byte past either end
    std::vector<uint8_t> out(cap ? cap : 1);
    int r = strom_zstd_host(7, z.data(), (uint32_t)z.size(), out.data(), cap);
    if (r != (int)cap || memcmp(out.data(), raw.data(), cap) != 0) {
      fprintf(stderr, "seed %s: status %d, want %u\n", argv[a], r, cap);
      return 1;
    }
    memset(out.data(), 0, out.size());
    r = strom_zstd_host_fp(7, z.data(), (uint32_t)z.size(), out.data(), cap, 4);
    if (r != (int)cap || memcmp(out.data(), raw.data(), cap) != 0) {
      fprintf(stderr, "seed %s (frame-parallel): status %d, want %u\n", argv[a], r, cap);
      return 1;
    }
    memset(out.data(), 0, out.size());
    r = lp1(z.data(), (uint32_t)z.size(), out.data(), cap);
    if (r != (int)cap || memcmp(out.data(), raw.data(), cap) != 0) {
      fprintf(stderr, "seed %s (lane-parallel): status %d, want %u\n", argv[a], r, cap);
      return 1;
    }
    ++ok;
    for (int i = 0; i < iters; ++i) {
      std::vector<uint8_t> m = z;
      const int kind = (int)(rng() % 3);
      if (kind == 2) {
        m.resize(rng() % m.size());
      } else {
        const int edits = 1 + (int)(rng() % 4);
        for (int e = 0; e < edits; ++e) {
          const size_t p = 4 + rng() % (m.size() - 4);
          if (kind == 0) m[p] = (uint8_t)rng();
          else m[p] ^= (uint8_t)(1u << (rng() % 8));
        }
      }
      uint8_t *in = (uint8_t *)malloc(m.size() ? m.size() : 1);
      memcpy(in, m.data(), m.size());
      r = strom_zstd_host(7, in, (uint32_t)m.size(), out.data(), cap);
      const int rf = strom_zstd_host_fp(7, in, (uint32_t)m.size(), out.data(), cap, 4);
      const int rl = lp1(in, (uint32_t)m.size(), out.data(), cap);
      free(in);
      if (rl != r) {
        fprintf(stderr, "lane-parallel status %d, serial %d\n", rl, r);
        return 1;
      }
      if (r > (int)cap || rf > (int)cap) {
        fprintf(stderr, "status %d / %d beyond the capacity %u\n", r, rf, cap);
        return 1;
      }
      if (r < 0) ++rejected;
      else ++decoded;
    }
  }
  printf("zstd_fuzz: %ld seeds ok, %ld mutants rejected, %ld decoded in range\n", ok, rejected,
         decoded);
  return 0;
}

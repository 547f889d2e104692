// Mutation test of the block-parallel LZ4 / snappy decoder's phases
// (csrc/kernels/lz4par.hip, host copy strom_lz4par_host: the same phase
// functions the GPU kernel runs — speculative walkers, scan-of-maps and
// round validation, serial walk, pointer fill / doubling), built host-only
// with ASan + UBSan (make build/lz4par_fuzz).  Every seed stream must
// decode to its reference output; random edits / truncations of it (byte
// flips, bit flips, a cut tail) must end in a clean status no larger than
// the capacity, never an out-of-range access.
//
//   lz4par_fuzz ITERATIONS CODEC SEED.bin SEED.raw [CODEC SEED.bin SEED.raw ...]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

extern "C" int strom_lz4par_host(int codec, const uint8_t *src, uint32_t src_len, uint8_t *dst,
                                 uint32_t cap, uint32_t *stats);

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
  if (argc < 5 || (argc - 2) % 3) {
    fprintf(stderr, "usage: %s ITERS CODEC SEED.bin SEED.raw ...\n", argv[0]);
    return 2;
  }
  const int iters = atoi(argv[1]);
  std::mt19937_64 rng(4321);
  long ok = 0, rejected = 0, decoded = 0, walked = 0;
  for (int a = 2; a < argc; a += 3) {
    const int codec = atoi(argv[a]);
    const std::vector<uint8_t> z = slurp(argv[a + 1]), raw = slurp(argv[a + 2]);
    if (z.size() < 16) return 2;
    const uint32_t cap = (uint32_t)raw.size();
    std::vector<uint8_t> out(cap ? cap : 1);   // exact size: ASan sees a byte past the end
    uint32_t st[8] = {0};
    int r = strom_lz4par_host(codec, z.data(), (uint32_t)z.size(), out.data(), cap, st);
    if (r != (int)cap || memcmp(out.data(), raw.data(), cap) != 0) {
      fprintf(stderr, "seed %s: status %d, want %u\n", argv[a + 1], r, cap);
      return 1;
    }
    walked += st[6] > 0;
    ++ok;
    for (int i = 0; i < iters; ++i) {
      std::vector<uint8_t> m = z;
      const int kind = (int)(rng() % 3);
      if (kind == 2) {
        m.resize(rng() % m.size());
      } else {
        const int edits = 1 + (int)(rng() % 4);
        for (int e = 0; e < edits; ++e) {
          const size_t p = 12 + rng() % (m.size() - 12);   // past the Arrow / frame header
          if (kind == 0) m[p] = (uint8_t)rng();
          else m[p] ^= (uint8_t)(1u << (rng() % 8));
        }
      }
      uint8_t *in = (uint8_t *)malloc(m.size() ? m.size() : 1);
      memcpy(in, m.data(), m.size());
      r = strom_lz4par_host(codec, in, (uint32_t)m.size(), out.data(), cap, st);
      free(in);
      if (r > (int)cap) {
        fprintf(stderr, "status %d beyond the capacity %u\n", r, cap);
        return 1;
      }
      if (r < 0) ++rejected;
      else ++decoded;
    }
  }
  printf("lz4par_fuzz: %ld seeds ok (%ld on walkers), %ld mutants rejected, %ld decoded in range\n",
         ok, walked, rejected, decoded);
  return 0;
}

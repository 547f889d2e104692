// Mutation test of strom_arrow_headers (csrc/engine/arrow_meta.cc), built
// with ASan + UBSan (make build/arrow_meta_fuzz): random byte edits of one
// valid record-batch header, written to a file and parsed; every outcome
// must be a clean return (0 or -EBADMSG), never an out-of-range access.
//
//   arrow_meta_fuzz FILE HEADER_OFFSET HEADER_LENGTH [ITERATIONS]
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <random>
#include <vector>

extern "C" int strom_arrow_headers(int, const int64_t *, int64_t, int32_t, int32_t, int64_t *,
                                   int32_t *, int32_t *, int32_t *, int64_t *, int64_t *, int32_t,
                                   int64_t *);

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s FILE OFFSET LENGTH [ITERS]\n", argv[0]);
    return 2;
  }
  const int64_t off = atoll(argv[2]), len = atoll(argv[3]);
  const int iters = argc > 4 ? atoi(argv[4]) : 20000;
  const int in = open(argv[1], O_RDONLY);
  if (in < 0 || len <= 0) return 2;
  std::vector<uint8_t> hdr(len);
  if (pread(in, hdr.data(), len, off) != len) return 2;
  close(in);
  const char *tmp = getenv("TMPDIR");
  std::string path = std::string(tmp ? tmp : "/tmp") + "/arrow_meta_fuzz.bin";
  std::mt19937 rng(1);
  int ok = 0, bad = 0;
  for (int it = 0; it < iters; ++it) {
    std::vector<uint8_t> b = hdr;
    const int nflip = 1 + (int)(rng() % 4);
    for (int j = 0; j < nflip; ++j) b[rng() % len] = (uint8_t)rng();
    const int fd = open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd < 0 || write(fd, b.data(), b.size()) != (ssize_t)b.size()) return 2;
    // also ask for more bytes than the file holds now and then
    int64_t blk[3] = {0, it % 7 == 0 ? len + 16 : len, 0};
    int64_t rows, nodes[8 * 2], bufs[16 * 2], badk;
    int32_t codec, nn, nb;
    const int rc = strom_arrow_headers(fd, blk, 1, 8, 16, &rows, &codec, &nn, &nb, nodes, bufs, 1,
                                       &badk);
    close(fd);
    if (rc == 0) {
      ++ok;
    } else if (rc == -EBADMSG && badk == 0) {
      ++bad;
    } else {
      fprintf(stderr, "unexpected rc %d (block %lld)\n", rc, (long long)badk);
      return 1;
    }
  }
  unlink(path.c_str());
  printf("arrow_meta_fuzz: %d parsed, %d rejected\n", ok, bad);
  return 0;
}

// sysprobe: checks which storage-path primitives are usable by an unprivileged
// process on this host (io_uring, O_DIRECT, FIEMAP, RWF_NOWAIT, mincore).
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <linux/fiemap.h>
#include <linux/fs.h>
#include <linux/io_uring.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/statfs.h>
#include <sys/syscall.h>
#include <sys/uio.h>
#include <unistd.h>

static void probe_dir(const char *dir) {
  char path[4096];
  snprintf(path, sizeof path, "%s/.sysprobe.%d", dir, getpid());
  struct statfs sf;
  if (statfs(dir, &sf) == 0)
    printf("[%s] f_type=0x%lx bsize=%ld\n", dir, (long)sf.f_type, (long)sf.f_bsize);
  int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0600);
  if (fd < 0) { printf("[%s] create failed: %s\n", dir, strerror(errno)); return; }
  size_t sz = 8 << 20;
  char *buf = aligned_alloc(4096, sz);
  memset(buf, 0x5a, sz);
  if (write(fd, buf, sz) != (ssize_t)sz) printf("[%s] write failed\n", dir);
  fsync(fd);
  // FIEMAP
  struct { struct fiemap fm; struct fiemap_extent ext[32]; } q;
  memset(&q, 0, sizeof q);
  q.fm.fm_length = ~0ULL; q.fm.fm_extent_count = 32; q.fm.fm_flags = FIEMAP_FLAG_SYNC;
  if (ioctl(fd, FS_IOC_FIEMAP, &q.fm) == 0) {
    printf("[%s] FIEMAP ok: %u extents", dir, q.fm.fm_mapped_extents);
    if (q.fm.fm_mapped_extents) printf(" first phys=%llu len=%llu flags=0x%x", (unsigned long long)q.ext[0].fe_physical, (unsigned long long)q.ext[0].fe_length, q.ext[0].fe_flags);
    printf("\n");
  } else printf("[%s] FIEMAP failed: %s\n", dir, strerror(errno));
  // RWF_NOWAIT
  struct iovec iov = {buf, 4096};
  ssize_t r = preadv2(fd, &iov, 1, 0, RWF_NOWAIT);
  printf("[%s] preadv2(RWF_NOWAIT) -> %zd (%s)\n", dir, r, r < 0 ? strerror(errno) : "ok");
  posix_fadvise(fd, 0, sz, POSIX_FADV_DONTNEED);
  void *m = mmap(NULL, sz, PROT_READ, MAP_SHARED, fd, 0);
  unsigned char vec[2048];
  if (m != MAP_FAILED && mincore(m, sz, vec) == 0) {
    int res = 0; for (size_t i = 0; i < sz / 4096; i++) res += vec[i] & 1;
    printf("[%s] mincore after DONTNEED: %d/%zu resident\n", dir, res, sz / 4096);
  }
  r = preadv2(fd, &iov, 1, 0, RWF_NOWAIT);
  printf("[%s] preadv2(RWF_NOWAIT) after DONTNEED -> %zd (%s)\n", dir, r, r < 0 ? strerror(errno) : "ok");
  close(fd);
  int dfd = open(path, O_RDONLY | O_DIRECT);
  if (dfd < 0) printf("[%s] O_DIRECT open failed: %s\n", dir, strerror(errno));
  else {
    r = pread(dfd, buf, 1 << 20, 0);
    printf("[%s] O_DIRECT pread 1MiB -> %zd (%s)\n", dir, r, r < 0 ? strerror(errno) : "ok");
    close(dfd);
  }
  unlink(path);
  free(buf);
}

int main(int argc, char **argv) {
  struct io_uring_params p;
  memset(&p, 0, sizeof p);
  int ring = syscall(__NR_io_uring_setup, 64, &p);
  if (ring < 0) printf("io_uring_setup: FAILED %s\n", strerror(errno));
  else { printf("io_uring_setup: ok features=0x%x sq_entries=%u\n", p.features, p.sq_entries); close(ring); }
  for (int i = 1; i < argc; i++) probe_dir(argv[i]);
  return 0;
}

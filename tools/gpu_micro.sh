#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
f=/tmp/strom_micro.bin
python - <<'PY'
import numpy as np, os
f="/tmp/strom_micro.bin"
rng=np.random.default_rng(1)
with open(f,"wb") as fh:
    for _ in range(16):
        fh.write(rng.integers(0,1<<63,size=(64<<20)//8,dtype=np.uint64).tobytes())
    os.fsync(fh.fileno())
fd=os.open(f,os.O_RDONLY); os.posix_fadvise(fd,0,0,os.POSIX_FADV_DONTNEED); os.close(fd)
PY
cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/shmem_enabled > gpurun_out/micro.log 2>&1
timeout -k 10 300 ./nvme_strom_amd/lib/strom_microbench $f 8 >> gpurun_out/micro.log 2>&1
echo "rc=$?"
HSA_ENABLE_SDMA=0 timeout -k 10 200 ./nvme_strom_amd/lib/strom_microbench > gpurun_out/micro_nosdma.log 2>&1
echo "rc=$?"
rm -f $f

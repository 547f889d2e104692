#!/bin/bash
# Decoder geometry sweep: lanes per stream (GL), history ring, input window.
# Correctness of the default build first; each variant is rebuilt on the box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "lz4 or snappy or malformed" > gpurun_out/pytest_dec.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
cp nvme_strom_amd/lib/libstrom.so /tmp/libstrom.default.so
for cfg in "4 2048 512" "4 1024 256" "4 2048 256" "2 1024 256" "2 512 256" "8 2048 512"; do
  set -- $cfg
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc/include -Icsrc/engine \
    -DSTROM_DECOMP_GL=${1}u -DSTROM_DECOMP_RING=${2}u -DSTROM_DECOMP_INW=${3}u \
    -c csrc/kernels/decompress.hip -o /tmp/decompress.o || exit 1
  objs=$(ls build/obj/engine/*.o build/obj/kernels/*.o | grep -v decompress.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o nvme_strom_amd/lib/libstrom.so $objs /tmp/decompress.o -lpthread -L/opt/rocm/lib -lrocprofiler-sdk-roctx -lhsa-runtime64 || exit 1
  echo "gl=$1 ring=$2 inw=$3"
  timeout -k 10 200 python -m nvme_strom_amd.tools.kbench --gib 1 --only lz4,snappy 2>&1 | grep decompress
  rc=$?; [ $rc -eq 0 ] || { echo "kbench rc=$rc"; cp /tmp/libstrom.default.so nvme_strom_amd/lib/libstrom.so; exit $rc; }
done
cp /tmp/libstrom.default.so nvme_strom_amd/lib/libstrom.so

set -o pipefail
for cfg in "4096 1024" "8192 2048"; do
  set -- $cfg
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc/include -Icsrc/engine -DSTROM_DECOMP_RING=${1}u -DSTROM_DECOMP_INW=${2}u -c csrc/kernels/decompress.hip -o build/obj/kernels/decompress.o && /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o nvme_strom_amd/lib/libstrom.so build/obj/engine/*.o build/obj/kernels/*.o -lpthread || exit 1
  echo "ring=$1 inw=$2"
  timeout -k 10 200 python -m nvme_strom_amd.tools.kbench --gib 1 --only lz4,snappy 2>&1 | grep -v "^{" | grep decompress
done

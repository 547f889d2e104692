set -o pipefail
mkdir -p gpurun_out/r3zgeo
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m nvme_strom_amd.tools.zstd_bench --libs ob1024,seq256,both --kinds val,ids,x,text --levels 1 --streams 2048,8192 --no-lz4 --out gpurun_out/r3zgeo/geo.json > gpurun_out/r3zgeo/geo.log 2>&1 && echo ok

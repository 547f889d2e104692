# same-process A/B of zstd decoder builds in nvme_strom_amd/lib/zv/ against
# the default library: bash tools/zgeo_ab.sh TAG LIB[,LIB...] [STREAMS]
set -o pipefail
TAG=${1:?tag}; LIBS=${2:?libs}; STREAMS=${3:-2048}
mkdir -p gpurun_out/$TAG
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m nvme_strom_amd.tools.zstd_bench --libs $LIBS --kinds val,ids,x,text --levels 1 \
  --streams $STREAMS --no-lz4 --out gpurun_out/$TAG/ab.json > gpurun_out/$TAG/ab.log 2>&1 && echo ok

#!/bin/bash
# GPU-box passes, run through gpurun from the repo root:
#   gpurun -- bash tools/gpu.sh TAG PHASE [PHASE...]
# Phases (each under its own time limit; the first failure ends the call):
#   tests      pytest -m gpu (one process)
#   ktests     GPU kernel numerics only (crc/heap/decoder/filter tests)
#   ztests     zstd decoder numerics only
#   zbench     zstd decoder GB/s by column kind / level / stream count (+ LZ4 rows)
#   zprof      zstd decoder phase profile (libstrom_zstdprof.so) by column kind
#   zpmc       two PMC passes (issue / wait / LDS / memory mix) over zstd_bench val + x
#   lppmc      the same over the LP zstd kernels only (--modes lp), summarized (pmc_summary)
#   lptrace    kernel trace + stats of the LP zstd kernels (time per kernel)
#   lzpmc      two PMC passes over the block-parallel LZ4 decoder (lz4par_bench), summarized
#   mvpmc      two PMC passes over the heap scan with / without the snapshot check (kbench mvcc)
#   zarrow     config-5 Arrow scan of a ZSTD-written file
#   ztrace     rocprofv3 kernel trace + stats of a short zstd_bench
#   zlibs      zstd decoder builds A/B (lib/zv/*.so, ZLIBS)
#   zgroups    Arrow ZSTD scan group count / read chunk / slots A/B (ZGROUPS)
#   zatrace    kernel trace of the Arrow ZSTD scan per group size (ingest grid vs decoder)
#   mtests     model-level GPU tests only (PG / Arrow / multi-rank scans)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (default flagship config)
#   kbench     per-kernel throughput (nvme_strom_amd.tools.kbench)
#   par        LZ4 decoder rows by stream count: lane groups vs block-parallel (lz4par)
#   dtests     decoder numerics tests only
#   ktrace     rocprofv3 kernel trace + stats of a short kbench
#   kpmc       one PMC pass (LDS / VALU / wave counters) over crc, heap, lz4
#   btrace     rocprofv3 kernel + memory-copy trace of a short bench run
#   sweep      block-size sweep 4K..4M vs the raw O_DIRECT ceiling
#   esweep     engine-only sweep (backend=cache) with per-worker attribution
#   lz4par     block-parallel LZ4 decoder by stream count (LZ4PAR_STREAMS / _KINDS / _ARGS)
#   dist       multi-rank Arrow / PG scans: 1 rank (RCCL) and 2 gloo ranks (DIST_ARGS)
#   overlap    load <-> side-stream collective overlap test + bench (priority and CU-masked grid streams)
#   otrace     rocprofv3 kernel trace of overlap_bench + grid/side concurrency summary
#   odtrace    the same with the zstd decoder as the side work (LDS co-residency)
#   benchtests bench.py contract tests (tests/test_gpu_bench.py)
#   ram        SSD2RAM (ssd2ram_test, 1 MiB units) vs the raw ceiling
#   decprof    decoder cycle profile per code path (libstrom_decprof.so)
#   decpmc     two PMC passes (issue / wait / LDS / memory instruction mix)
#              over the LZ4 decoder build DECLIB (default lib/ab/base.so)
#   arrow      config-5 Arrow scan bench (tools.arrow_bench)
#   ceiling    engine + ingest ceiling: page-cache reads (backend=cache) vs O_DIRECT
#   pg         end-to-end PostgreSQL heap scan (GPU ring vs the reference-shaped CPU scan)
#   stripe     config-3 proxy: 4-member stripe set vs one file (tools.stripe_bench)
#   probe      Arrow column reads alone vs storage_seq and vs the same requests read raw
#              (tools.arrow_read_probe; PROBE_ARGS)
#   benchab    bench.py arms alternated round by round, each with its own STROM_* settings:
#              BENCHAB="def: lifo:SLOT_LIFO=1 s6:STAGING_SLOTS=6,QUEUE_DEPTH=8" BENCHAB_ROUNDS=3
#              (how every staging / geometry A/B of profiles/r6/SUMMARY.md was run)
# Output lands in gpurun_out/TAG/.  One-off recipes (several phases with
# env overrides) live in tools/run/, which git ignores; the commands behind
# every committed profile are written into its profiles/rN/*/SUMMARY.md.
set -o pipefail
TAG=${1:?tag}; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export PYTHONPATH=$PWD${PYTHONPATH:+:$PYTHONPATH}
ROOT=$PWD
step() {
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -40 "$OUT/$name.log"; exit $rc; fi
}
for phase in "$@"; do
  case $phase in
    tests) step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    ktests) step ktests 300 python -u -m pytest tests/test_gpu_core.py tests/test_gpu_kernels.py -m gpu -x -q \
              --timeout 120 --timeout-method thread -k "crc or heap or lz4 or snappy or malformed or filter or compact" ;;
    ztests) step ztests 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v \
              --timeout 120 --timeout-method thread -k zstd ;;
    mtests) step mtests 300 python -u -m pytest tests/test_gpu_models.py -m gpu -x -v \
              --timeout 120 --timeout-method thread ;;
    smoke) step smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 400 python bench.py; grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"; cat "$OUT/bench.json" ;;
    kbench) step kbench 300 python -u -m nvme_strom_amd.tools.kbench --out "$OUT/kbench.json" ;;
    zbench) step zbench 300 python -u -m nvme_strom_amd.tools.zstd_bench --out "$OUT/zstd.json" ;;
    zprof) step zprof 300 python -u -m nvme_strom_amd.tools.zstd_bench --prof --no-lz4 --streams ${ZSTREAMS:-2048} --out "$OUT/zprof.json" ;;
    zpmc) for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
                      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
            n=$((n + 1))
            (cd /tmp && step zpmc$n 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/zpmc$n" -o pmc \
              -- python3 -m nvme_strom_amd.tools.zstd_bench --kinds ${ZKINDS:-val,x} --levels 1 --streams ${ZSTREAMS:-2048} --modes ${ZMODES:-auto} \
                 --no-lz4 --iters 1) || exit 1
          done ;;
    lppmc) n=0 # the LP zstd decoder's kernels (walk / lit / seq / exec / serial): two PMC passes
          for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
                      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
            n=$((n + 1))
            (cd /tmp && step lppmc$n 120 rocprofv3 --pmc $pass --kernel-include-regex zstd_lp --output-format csv \
              -d "$OUT/lppmc$n" -o pmc -- python3 -m nvme_strom_amd.tools.zstd_bench --kinds ${ZKINDS:-val,ids,text} \
                 --levels 1 --streams ${ZSTREAMS:-2048} --modes lp --no-lz4 --iters 1) || exit 1
          done
          step lppmcsum 60 python3 -m nvme_strom_amd.tools.pmc_summary "$OUT"/lppmc1 "$OUT"/lppmc2 \
            --out "$OUT/lppmc_summary.json" ;;
    lptrace) # per-kernel device time of the LP zstd decoder (walk / lit / seq / exec / serial)
          (cd /tmp && step lptrace 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lptrace" -o trace \
            -- python3 -m nvme_strom_amd.tools.zstd_bench --kinds ${ZKINDS:-val,ids,text} --levels 1 \
               --streams ${ZSTREAMS:-2048} --modes lp --no-lz4 --iters 3) || exit 1 ;;
    lzpmc) n=0 # the block-parallel LZ4 decoder (lz4par_kernel_*): two PMC passes, summarized
          for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
                      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
            n=$((n + 1))
            (cd /tmp && step lzpmc$n 120 rocprofv3 --pmc $pass --kernel-include-regex lz4par_kernel --output-format csv \
              -d "$OUT/lzpmc$n" -o pmc -- python3 -m nvme_strom_amd.tools.lz4par_bench --kinds ${LZKINDS:-val,ids,text} \
                 --streams ${LZSTREAMS:-2048} --distinct 32 --iters 1 --no-lanes) || exit 1
          done
          step lzpmcsum 60 python3 -m nvme_strom_amd.tools.pmc_summary "$OUT"/lzpmc1 "$OUT"/lzpmc2 \
            --out "$OUT/lzpmc_summary.json" ;;
    mvpmc) n=0 # the heap scan's snapshot-check instance vs the plain one: two PMC passes over kbench mvcc
          for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
                      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
            n=$((n + 1))
            (cd /tmp && step mvpmc$n 120 rocprofv3 --pmc $pass --kernel-include-regex heap_scan --output-format csv \
              -d "$OUT/mvpmc$n" -o pmc -- python3 -m nvme_strom_amd.tools.kbench --gib 0.5 --only mvcc) || exit 1
          done
          step mvpmcsum 60 python3 -m nvme_strom_amd.tools.pmc_summary "$OUT"/mvpmc1 "$OUT"/mvpmc2 \
            --out "$OUT/mvpmc_summary.json" ;;
    zarrow) step zarrow 400 python -u -m nvme_strom_amd.tools.arrow_bench --codec zstd --out "$OUT/arrow_zstd.json" ;;
    zlibs) # same-process A/B of zstd decoder builds in nvme_strom_amd/lib/zv/ (ZLIBS=a,b ZSTREAMS=...)
          step zlibs 400 python -u -m nvme_strom_amd.tools.zstd_bench --libs ${ZLIBS:?ZLIBS} --kinds val,ids,x,text \
            --levels 1 --streams ${ZSTREAMS:-2048} --no-lz4 --out "$OUT/zlibs.json" ;;
    zgroups) # Arrow ZSTD scan: group count x read chunk x slots, arms in one call (ZGROUPS="div:chunk_kib:nslots ...")
          for arm in ${ZGROUPS:-1:64:3 2:16:4 1:16:3}; do
            IFS=: read -r dv ck ns <<< "$arm"
            STROM_ARROW_ZSTD_DIV=$dv step zg_${dv}_${ck}_${ns} 300 python -u -m nvme_strom_amd.tools.arrow_bench --codec zstd \
              --columns val --no-strings --reps ${ZREPS:-7} --chunk-kib $ck --nslots $ns --slot-mib 1024 \
              --out "$OUT/zg_${dv}_${ck}_${ns}.json"
          done ;;
    zatrace) # kernel trace of the Arrow ZSTD scan at ZATRACE_DIVS group sizes: ingest grid vs decoder concurrency
          for dv in ${ZATRACE_DIVS:-1 4}; do
            (cd /tmp && STROM_ARROW_ZSTD_DIV=$dv step zatrace_d$dv 300 rocprofv3 --kernel-trace --stats --output-format csv \
              -d "$OUT/zatrace_d$dv" -o trace -- python3 -m nvme_strom_amd.tools.arrow_bench --codec zstd --columns val \
              --no-qual2 --no-strings --reps 2 --out "$OUT/zatrace_d$dv.json") || exit 1
            python -m nvme_strom_amd.tools.overlap_trace $(find "$OUT/zatrace_d$dv" -name '*kernel_trace.csv' | head -1) \
              --side zstd --md "$OUT/zatrace_d${dv}_summary.md" > "$OUT/zatrace_d${dv}_summary.txt" 2>&1 || exit 1
          done ;;
    ztrace) (cd /tmp && step ztrace 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ztrace" -o trace \
              -- python3 -m nvme_strom_amd.tools.zstd_bench --kinds val,x --levels 1 --streams 2048 --no-lz4) ;;
    par) step par 300 python -u -m nvme_strom_amd.tools.kbench --only par --out "$OUT/par.json" ;;
    dtests) step dtests 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q \
              --timeout 120 --timeout-method thread -k "lz4 or snappy or malformed or geometr" ;;
    ktrace) (cd /tmp && step ktrace 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o trace \
              -- python3 -m nvme_strom_amd.tools.kbench --gib 0.5) ;;
    kpmc) (cd /tmp && step kpmc 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
              SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$OUT/pmc" -o pmc \
              -- python3 -m nvme_strom_amd.tools.kbench --gib 0.5 --only crc,heap,lz4) ;;
    btrace) (cd /tmp && step btrace 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/btrace" -o btrace \
              -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --lat-samples 300) ;;
    esweep) # engine-only sweep with worker phase attribution; ESWEEP_NAME / ESWEEP_ARGS
            nm=${ESWEEP_NAME:-esweep}
            step $nm 500 python -u -m nvme_strom_amd.tools.sweep --engine-only --prof --no-lat \
              --blocks ${SWEEP_BLOCKS:-4K,8K,16K} ${ESWEEP_ARGS:-} --out "$OUT/$nm.json" ;;
    lz4par) step lz4par 500 python -u -m nvme_strom_amd.tools.lz4par_bench --kinds ${LZ4PAR_KINDS:-val,ids,text} \
              --streams ${LZ4PAR_STREAMS:-512,2048,8192} --distinct 32 --iters 5 ${LZ4PAR_ARGS:-} --out "$OUT/lz4par.json" ;;
    dist) # multi-rank scan (parallel/scan.py): 1 rank RCCL, 2 ranks gloo on the one GPU; DIST_ARGS
          step dist1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
            --master-port 29561 -m nvme_strom_amd.tools.dist_scan_bench ${DIST_ARGS:---rows 134217728} --reps 3 \
            --out "$OUT/dist1.json"
          step dist2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
            --master-port 29562 -m nvme_strom_amd.tools.dist_scan_bench ${DIST_ARGS:---rows 134217728} --reps 3 \
            --backend gloo --out "$OUT/dist2_gloo.json" ;;
    overlap) step otests 300 python -u -m pytest tests/test_gpu_overlap.py -m gpu -x -v --timeout 200 --timeout-method thread
             step overlap 300 python -u -m nvme_strom_amd.tools.overlap_bench --window-mib 256 --steps 12 --calibrate \
               --n 2,8 --out "$OUT/overlap.json"
             step overlap_dec 300 python -u -m nvme_strom_amd.tools.overlap_bench --window-mib 512 --steps 6 --calibrate \
               --side decode --n 2 --out "$OUT/overlap_dec.json"
             STROM_INGEST_PRIO=0 step overlap_cumask 300 python -u -m nvme_strom_amd.tools.overlap_bench --window-mib 256 --steps 12 \
               --gather-reps ${OV_REPS:-8} --n 2,8 --out "$OUT/overlap_cumask.json" ;;
    odtrace) # the ingest grid next to the LDS-heavy zstd decoder: kernel trace + concurrency summary
            (cd /tmp && step odtrace 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/odtrace" -o trace \
              -- python3 -m nvme_strom_amd.tools.overlap_bench --side decode --calibrate --n 2 --modes overlap --window-mib 512 --steps 6 \
                 --out "$OUT/odtrace.json") && \
            python -m nvme_strom_amd.tools.overlap_trace $(find "$OUT/odtrace" -name '*kernel_trace.csv' | head -1) \
              --side zstd --md "$OUT/odtrace_summary.md" ;;
    otrace) (cd /tmp && step otrace 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/otrace" -o trace \
              -- python3 -m nvme_strom_amd.tools.overlap_bench --window-mib 256 --steps 8 --gather-reps ${OV_REPS:-8} --n 8 --modes overlap) && \
            python -m nvme_strom_amd.tools.overlap_trace $(find "$OUT/otrace" -name '*kernel_trace.csv' | head -1) \
              --md "$OUT/otrace_summary.md" ;;
    benchtests) step benchtests 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench.py ;;
    sweep) step sweep 400 python -u -m nvme_strom_amd.tools.sweep --out "$OUT/sweep.json" ;;
    ram) step ram 500 python -u -m nvme_strom_amd.tools.ram_bench --file-gib ${RAM_GIB:-8} --reps ${RAM_REPS:-7} --out "$OUT/ram.json" ;;
    decprof) step decprof 300 python -u -m nvme_strom_amd.tools.decomp_prof --out "$OUT/decprof.json" ;;
    decpmc) for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
                        "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"; do
              n=$((n + 1))
              (cd /tmp && step decpmc$n 90 rocprofv3 --pmc $pass --output-format csv -d "$OUT/decpmc$n" -o pmc \
                -- python3 -m nvme_strom_amd.tools.decomp_ab "$ROOT/${DECLIB:-nvme_strom_amd/lib/ab/base.so}" \
                   --rounds 1 --cases "${DECCASES:-lz4_words,lz4_ints}") || exit 1
            done ;;
    probe) step probe 600 python -u -m nvme_strom_amd.tools.arrow_read_probe ${PROBE_ARGS:---codec zstd --columns val,x} \
             --out "$OUT/probe.json" ;;
    benchab) i=0
      for r in $(seq 1 ${BENCHAB_ROUNDS:-2}); do
        for arm in ${BENCHAB:-def:}; do
          i=$((i + 1)); name=${arm%%:*}; kv=${arm#*:}; envs=()
          for x in ${kv//,/ }; do envs+=("STROM_$x"); done
          step "bench_${i}_$name" 300 env "${envs[@]}" python -u bench.py
          grep '^{' "$OUT/bench_${i}_$name.log" | tail -1 > "$OUT/bench_${i}_$name.json"
        done
      done ;;
    pg) step pg 400 python -u -m nvme_strom_amd.tools.pg_bench --out "$OUT/pg.json" ;;
    stripe) step stripe 400 python -u -m nvme_strom_amd.tools.stripe_bench --out "$OUT/stripe.json" ;;
    ceiling) step ceiling 400 python -u -m nvme_strom_amd.tools.ceiling_bench --out "$OUT/ceiling.json" ;;
    arrow) step arrow 700 python -u -m nvme_strom_amd.tools.arrow_bench --out "$OUT/arrow.json" ;;
    *) echo "unknown phase $phase"; exit 2 ;;
  esac
done
echo done

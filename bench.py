#!/usr/bin/env python3
"""Headline benchmark: SSD→GPU read GiB/s + p50 4 KiB IOP latency.

One process per GPU (torchrun for N>1, RCCL over xGMI; ``--gpus N`` run
outside torchrun starts a child torchrun with N ranks and relays rank 0's
line, so ``n_gpus`` is always the number of ranks that ran).  Each rank owns a
synthetic random-byte shard file; a *step* loads a ``--window-mib`` window of
its shard into a resident HBM buffer through the engine (MEMCPY_SSD2GPU,
nvme_test methodology: 32 MiB segments of 8 KiB chunks, 6 segments in
flight — reference utils/nvme_test.c:40-41, 301-302, 383-498).  With N>1 the
previous step's shard is all-gathered over RCCL on a side stream while the
next window loads (parallel/fanout.ShardedLoader: status word + data
collective per step, failure consensus, per-slice CRC check of the last
fan-out).  ``value`` = total bytes loaded by all ranks / max-rank
wall time (GiB/s, weak scaling).  Also reported: p50/p99 latency of single
4 KiB reads into HBM (QD1), the VFS control (pread → pinned → HtoD, the
reference's ``nvme_test -f``) and a CRC32C check of the last window on the
GPU against the host CRC of the file.

``vs_baseline`` = value / VFS control measured in the same run: the reference
publishes no numbers, its methodology's control is the
baseline to beat on this machine.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

METRIC = "SSD→GPU read GiB/s + p50 4KiB IOP latency at 1/2/4/8 MI355X"


def _log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def make_shard(path: str, nbytes: int, seed: int) -> None:
    if os.path.exists(path) and os.path.getsize(path) == nbytes:
        return
    rng = np.random.default_rng(seed)
    piece = 64 << 20
    with open(path + ".tmp", "wb") as f:
        left = nbytes
        while left:
            n = min(piece, left)
            f.write(rng.integers(0, 1 << 63, size=n // 8, dtype=np.uint64).tobytes())
            left -= n
        f.flush()
        os.fsync(f.fileno())
    os.replace(path + ".tmp", path)


def shard_bytes(want: int, window: int, free: int, have: int, local_world: int) -> int:
    """Shard size per rank: ``want`` capped at 80 % of the directory's free
    space (plus this rank's existing shard) split over the node's ranks, in
    whole windows, never below one window."""
    cap = int((free + have) * 0.8) // max(1, local_world) // window * window
    return min(want, max(cap, window))


def fs_type(path: str) -> str:
    """Filesystem type of the mount holding ``path`` (longest mountinfo prefix)."""
    best, typ = "", "unknown"
    real = os.path.realpath(path)
    try:
        with open("/proc/self/mountinfo") as f:
            for line in f:
                parts = line.split()
                mnt = parts[4]
                fst = parts[parts.index("-") + 1]
                if (real == mnt or real.startswith(mnt.rstrip("/") + "/")) and len(mnt) > len(best):
                    best, typ = mnt, fst
    except OSError:
        pass
    return typ


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv: list) -> int:
    """``--gpus N`` outside torchrun: run N ranks as a CHILD torchrun (never
    exec: this process has not touched the GPU and stays the parent), relay
    its output, and fail unless rank 0 printed a result line for N ranks."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + argv
    print("[bench] launching", " ".join(cmd[1:]), file=sys.stderr, flush=True)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    result = None
    for line in p.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
        if line.startswith("{"):
            try:
                result = json.loads(line)
            except ValueError:
                pass
    rc = p.wait()
    if rc != 0:
        return rc
    if result is None or result.get("n_gpus") != n:
        print(f"[bench] child run printed no result for {n} ranks", file=sys.stderr)
        return 1
    return 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--window-mib", type=int, default=1024, help="bytes loaded per rank per step")
    ap.add_argument("--file-gib", type=float, default=4.0, help="shard file size per rank")
    ap.add_argument("--segment-mib", type=int, default=32)
    ap.add_argument("--depth", type=int, default=6, help="segments in flight")
    ap.add_argument("--chunk", type=int, default=8192)
    ap.add_argument("--lat-samples", type=int, default=2000)
    ap.add_argument("--fanout", choices=["allgather", "broadcast", "none"], default="allgather")
    ap.add_argument("--dir", default=os.environ.get("STROM_BENCH_DIR", "/tmp/strom_bench"))
    ap.add_argument("--keep", action="store_true", help="keep shard files")
    ap.add_argument("--no-verify-each", dest="verify_each", action="store_false",
                    help="N > 1: skip the per-step device CRC of every gathered slice")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group backend (nccl = RCCL; gloo rehearses the multi-rank "
                         "path with several ranks on one GPU, collectives staged via the host)")
    a = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a.gpus, sys.argv[1:])

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {a.gpus}")

    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
    if a.backend == "nccl" and local_world > ndev:
        raise SystemExit(f"bench: {local_world} ranks on this node but {ndev} GPUs visible "
                         "(RCCL needs one GPU per rank; --backend gloo rehearses on one GPU)")
    # gloo rehearsal: ranks beyond the visible GPUs share them
    local_dev = local % max(1, ndev)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == a.gpus
    # small control-plane collectives: device tensors under RCCL, host under gloo
    cdev = dev if a.backend == "nccl" else torch.device("cpu")

    def allreduce(vals, op):
        t = torch.tensor(vals, dtype=torch.float64, device=cdev)
        if world > 1:
            dist.all_reduce(t, op=op)
        return t.tolist()

    import nvme_strom_amd as S
    from nvme_strom_amd.models.ssd2gpu_stream import vfs_control
    from nvme_strom_amd.parallel.fanout import ShardedLoader

    os.makedirs(a.dir, exist_ok=True)
    W = a.window_mib << 20
    F = int(a.file_gib * (1 << 30)) // W * W
    F = max(F, W)
    path = os.path.join(a.dir, f"shard_r{rank}.bin")
    # every rank of the node writes its shard to the same directory: size the
    # shards to 80 % of the free space (same size on every rank: MIN over
    # ranks, taken before anyone writes), never below one window
    import shutil
    have = os.path.getsize(path) if os.path.exists(path) else 0
    F = shard_bytes(F, W, shutil.disk_usage(a.dir).free, have, local_world)
    F = int(allreduce([F], dist.ReduceOp.MIN if world > 1 else None)[0])
    t0 = time.time()
    make_shard(path, F, 1234 + rank)
    # reader pool per rank: split only among ranks that share this shard's
    # backing device (placement.plan_io all-gathers the device identities)
    from nvme_strom_amd.parallel.placement import plan_io
    placement = plan_io(path, device=local_dev)
    _log(rank, f"placement {placement}")
    fd = os.open(path, os.O_RDONLY)
    S.evict_file(fd)
    _log(rank, f"shard {F >> 20} MiB ready in {time.time() - t0:.1f}s, resident="
               f"{S.resident_bytes(fd) >> 20} MiB, engine={S.version()} provider={S.provider()}")

    fstype = fs_type(a.dir)
    mode = a.fanout if world > 1 else "none"
    fan = mode != "none"
    # the loader: window i of this rank's shard into HBM buffer i % 2 while
    # the side stream fans out window i-1 (status word + RCCL all-gather)
    # N > 1: every step's gathered shards are delivered to a consumer on the
    # loader's consumer stream (on_gathered, after the step's gather, while
    # the next window loads) and every slice is CRC-checked on the device
    # against its source rank's CRC of the window as it landed
    # (verify_each) — inside the timed loop: the check's device time is
    # reported (per_rank.slice_check_ms_per_rank)
    delivered = {"steps": 0, "bytes": 0}

    def consume(g):
        delivered["steps"] += 1
        delivered["bytes"] += g.tensor.numel()

    ld = ShardedLoader(path, W, dev, mode=mode, segment_sz=a.segment_mib << 20,
                       chunk_sz=a.chunk, depth=a.depth, out_ring=2,
                       on_gathered=consume if fan else None, verify_each=fan and a.verify_each)
    nwin = ld.nwin

    # the storage's own sequential rate (below), once before the timed loop
    # as well as after it: the better of the two is the ceiling
    mreq = int(S.config_get("max_request"))
    nw, qd = int(S.config_get("workers")), int(S.config_get("queue_depth"))

    def storage_seq() -> dict:
        if world > 1:
            dist.barrier()
        # into plain pages and into registered 2 MiB-page buffers
        # (READ_FIXED, as the engine's pinned staging)
        return {("fixed" if fx else "plain"): S.raw_read_rate(
            fd, mreq, max(64, 4 * W // mreq), threads=nw, qd=min(256, max(1, qd)),
            sequential=True, fixed=fx)[1] for fx in (False, True)}

    seq_pre = storage_seq()
    for i in range(a.warmup):
        ld.step(i)
    ld.flush()
    ld.stats = type(ld.stats)()
    ld.gather_seconds()
    ld.gather_s = 0.0
    ld.crc_seconds()
    ld.crc_s = 0.0
    delivered.update(steps=0, bytes=0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        ld.step(a.warmup + i)
    ld.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0

    # max over ranks
    tmax = allreduce([dt], dist.ReduceOp.MAX if world > 1 else None)[0]
    total_bytes = world * W * a.steps
    value = total_bytes / tmax / (1 << 30)
    per_rank = ld.report(wall_s=dt)
    st = ld.stats
    agg = dict(nr_ram=st.nr_ram, nr_ssd=st.nr_ssd, nr_submit=st.nr_submit, nr_blocks=st.nr_blocks)

    # integrity of the last loaded window, and of every slice of the last
    # fan-out (collective CRC check, not timed)
    last = a.warmup + a.steps - 1
    verified = ld.verify(last)
    gather_ok = verified if fan else None
    buf = ld.bufs[last % len(ld.bufs)]

    # QD1 4 KiB reads into HBM (O_DIRECT path), timed in the engine's native
    # loop (the reference's C-tool vantage).  The headline reads go through a
    # registered file (RegisteredFile: the descriptor resolved once, as the
    # reference's module holds the file for an ioctl) and alternate read by
    # read with raw O_DIRECT preads of other offsets (order flipped every
    # pair), so the storage floor they are compared with is the same
    # moment's.  A plain descriptor's numbers (a kcmp identity check per
    # read) and the Python-binding probe are reported alongside.
    nan = float("nan")
    lat = lat_plain = lat_py = np.array([nan])
    phases, phases_plain, paired, raw_p50, floor = {}, {}, {}, nan, nan

    def pair(rfd, n):
        S.evict_file(fd)
        offs = rng.integers(0, F // 4096, size=2 * (n + 50)) * 4096
        pe, pr = (x[50:].astype(np.float64) / 1e3 for x in S.pread_pair_latency(buf.handle, 0, rfd, offs))
        return pe, pr, {"engine_p50_us": round(float(np.median(pe)), 2),
                        "raw_p50_us": round(float(np.median(pr)), 2),
                        "overhead_p50_us": round(float(np.median(pe - pr)), 2),
                        "pairs": int(len(pe))}

    def phase_split(rfd, n):
        S.evict_file(fd)
        offs = rng.integers(0, F // 4096, size=n + 50) * 4096
        return S.phase_breakdown(S.pread_gpu_phases(buf.handle, 0, rfd, offs)[50:])

    if a.lat_samples:
        rng = np.random.default_rng(rank)
        S.stat_hist(reset=True)
        with S.RegisteredFile(fd) as rf:
            lat, pr, paired = pair(rf.fd, a.lat_samples)
            floor = float(np.median(pr))
            paired["note"] = ("registered file; raw O_DIRECT pread and pread_gpu alternated read "
                              "by read, order flipped every pair; overhead = median of pairwise "
                              "differences")
            phases = phase_split(rf.fd, min(a.lat_samples, 1000))
        _, _, paired["plain_descriptor"] = pair(fd, min(a.lat_samples, 1000))
        phases_plain = phase_split(fd, min(a.lat_samples, 1000))
        S.evict_file(fd)
        offs = rng.integers(0, F // 4096, size=min(a.lat_samples, 1000) + 50) * 4096
        lat_plain = S.pread_gpu_latency(buf.handle, 0, fd, offs)[50:] / 1e3
        # the floor in a pass of its own (the round-4 vantage)
        S.evict_file(fd)
        raw_p50 = float(np.percentile(S.pread_raw_latency(fd, offs)[50:], 50)) / 1e3
        S.evict_file(fd)
        offs = rng.integers(0, F // 4096, size=min(a.lat_samples, 500) + 50) * 4096
        py = []
        for j, off in enumerate(offs.tolist()):
            t1 = time.perf_counter_ns()
            S.pread_gpu(buf.handle, 0, fd, off, 4096)
            t2 = time.perf_counter_ns()
            if j >= 50:
                py.append((t2 - t1) / 1e3)
        lat_py = np.array(py)
    p50, p99 = float(np.percentile(lat, 50)), float(np.percentile(lat, 99))
    p50_plain = float(np.percentile(lat_plain, 50))
    p50_py = float(np.percentile(lat_py, 50))

    # the same QD1 reads through the v0.6 ioctl pair (SSD2GPU + WAIT: task
    # table, residency probe, planner), and the host primitive costs below both
    ioctl_p50 = float("nan")
    costs = {}
    if a.lat_samples:
        S.evict_file(fd)
        offs = rng.integers(0, F // 4096, size=min(a.lat_samples, 1000) + 50) * 4096
        ioctl_p50 = float(np.percentile(S.ioctl_latency(buf.handle, 0, fd, offs)[50:], 50)) / 1e3
        costs = S.host_costs(fd)
        costs.update({"engine_" + k: v for k, v in S.engine_costs(buf.handle, fd).items()})

    # the storage's own sequential rate in this run: host-only io_uring
    # O_DIRECT reads of the same shard, the engine's request size, ring
    # count and depth, each ring over its own run of the file (no GPU, no
    # engine) — so value / storage says how much of the storage the load
    # path delivers.  All ranks read at once, as their loads do.
    seq_post = storage_seq()
    seq_modes = {f"{k}_{when}": v for when, m in (("before", seq_pre), ("after", seq_post))
                 for k, v in m.items()}
    seq_gib = max(seq_modes.values())
    # VFS control: pread -> pinned -> HtoD, same window
    S.evict_file(fd)
    vt = vfs_control(path, 0, W, buf.tensor, segment_sz=a.segment_mib << 20, nr_segments=a.depth)
    vfs = W / vt / (1 << 30)
    # worst rank for latencies, sum of ranks for the control's throughput
    if world > 1:
        p50, p99, p50_py, ioctl_p50, p50_plain, floor = allreduce(
            [p50, p99, p50_py, ioctl_p50, p50_plain, floor], dist.ReduceOp.MAX)
        vfs_total = allreduce([vfs], dist.ReduceOp.SUM)[0]
        seq_total = allreduce([seq_gib], dist.ReduceOp.SUM)[0]
        seq_modes = dict(zip(seq_modes, allreduce(list(seq_modes.values()), dist.ReduceOp.SUM)))
    else:
        vfs_total = vfs
        seq_total = seq_gib
    ver = 1.0 if verified else 0.0
    hist = S.stat_hist()
    ing = S.ingest_info(local_dev)
    steps_bytes = (a.warmup + a.steps) * W
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(tmax / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / vfs_total, 3) if vfs_total > 0 else None,
        "baseline": "VFS control (pread->pinned->HtoD, nvme_test -f methodology) on the same box",
        "vfs_control_GiBps": round(vfs_total, 3),
        "storage_seq_GiBps": round(seq_total, 3),
        "of_storage": round(value / seq_total, 3) if seq_total > 0 else None,
        "storage_seq_note": (f"host-only io_uring O_DIRECT sequential read of the same shard, "
                             f"{mreq >> 10} KiB requests, {nw} rings x QD {qd}, disjoint run per "
                             "ring, all ranks at once, same run; the best of plain and "
                             "registered 2 MiB-page buffers, before and after the timed loop"),
        "storage_seq_modes_GiBps": {k: round(v, 3) for k, v in seq_modes.items()},
        "p50_4k_lat_us": round(p50, 2),
        "p99_4k_lat_us": round(p99, 2),
        "p50_4k_lat_python_us": round(p50_py, 2),
        "p50_4k_lat_plain_fd_us": round(p50_plain, 2),
        "p50_4k_lat_note": ("p50/p99: QD1 4 KiB pread_gpu through a registered file, alternated "
                            "read by read with raw O_DIRECT preads (storage_4k_p50_us is their "
                            "median: the floor at the same moment); plain_fd: a plain "
                            "descriptor, native loop; raw_odirect: the floor in a pass of its own"),
        "p50_4k_lat_ioctl_us": round(ioctl_p50, 2),
        "host_costs_ns": costs,
        "engine_io_p50_us": round(S.hist_percentile(hist["io_ns"], 50) / 1e3, 2),
        "raw_odirect_4k_p50_us": round(raw_p50, 2),
        "storage_4k_p50_us": round(floor, 2),
        "storage": {
            "fs_type": fstype,
            "dir": a.dir,
            "path": ("P2P: NVMe READ -> HBM BAR (kernel provider)" if S.provider() == "kernel" else
                     "host-bounce (userspace provider): O_DIRECT read -> pinned staging -> "
                     + ("GPU ingest grid" if ing and ing["available"] else "SDMA copy") + " -> HBM"),
            "note": ("backing store answers 4 KiB O_DIRECT reads in "
                     f"{raw_p50:.1f} us: RAM-class, not NAND"
                     if raw_p50 == raw_p50 and raw_p50 < 20 else "device-class latency"),
            "file_bytes_per_rank": F,
            "bytes_read_per_rank": steps_bytes,
            "windows_reread": max(0, (a.warmup + a.steps) - nwin),
            "reread_note": "O_DIRECT: a re-read window is read from the backing store again "
                           "(no page cache in the path)",
        },
        "rccl": {"world_size": dist.get_world_size() if world > 1 else 1,
                 "backend": dist.get_backend() if world > 1 else None,
                 "collective": mode, "staged_via_host": ld.staged,
                 "allgather_verified": gather_ok,
                 "delivered_steps": delivered["steps"], "delivered_bytes": delivered["bytes"],
                 "per_step_slice_check": bool(fan and a.verify_each)},
        "per_rank": per_rank,
        "latency_reduction": "max over ranks (worst rank)",
        "ingest_grid": ing,
        "p50_4k_phases_us": phases,
        "p50_4k_phases_plain_fd_us": phases_plain,
        "qd1_paired": paired,
        "verified_crc32c": bool(ver == 1.0),
        "avg_request_kib": round(0.5 * agg["nr_blocks"] / agg["nr_submit"], 1) if agg["nr_submit"] else 0,
        "ram_chunks": agg["nr_ram"],
        "ssd_chunks": agg["nr_ssd"],
        "dtype": "uint8",
        "data": "synthetic random-byte shard file per rank (O_DIRECT reads)",
        "config": {
            "model": f"ssd2gpu_stream(segment={a.segment_mib}MiB x depth {a.depth}, chunk={a.chunk}B)",
            "global_batch": world * W,
            "seq_len": a.chunk,
            "parallelism": f"dp{world}" + (f"+{mode}" if fan else ""),
            "window_bytes_per_rank": W,
            "file_bytes_per_rank": F,
            "backend": S.config_get("backend"),
            "workers": int(S.config_get("workers")),
            "placement": placement,
            "max_request": int(S.config_get("max_request")),
            "engine": {k: S.config_get(k) for k in ("queue_depth", "staging_slots", "stage_by_bytes",
                                                     "slot_lifo", "ingest", "ingest_grid",
                                                     "ingest_piece", "fixed_bufs")},
        },
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ld.close()
    os.close(fd)
    if not a.keep:
        try:
            os.unlink(path)
        except OSError:
            pass
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

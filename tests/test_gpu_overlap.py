"""Load <-> side-stream overlap on one GPU.

The fan-out schedule (parallel/fanout.py) runs step i's all-gather on a side
stream while step i+1 loads through the engine's persistent ingest grid.
Here the collective is replaced by CU copy kernels on a side stream sized
like an N-rank all-gather's receive traffic, or by the lane-parallel zstd
decoder (LDS-heavy: the co-residency an Arrow ZSTD scan's read / decode
overlap needs) — nvme_strom_amd/tools/overlap_bench.py.  The side work is
calibrated to about half a load on the box at hand; the fanout.report()
overlap formula must show it hidden behind the loads, and the loads must
not get slower while it runs (else the formula would read high for the
wrong reason)."""
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import nvme_strom_amd as S
    S.configure(gpu_emulation=0)
    return S


def _hidden(r):
    """The share of the shorter of (loads, side work) hidden behind the
    other: fanout.report()'s formula when the side work is the shorter."""
    return (r["load_s"] + r["gather_s"] - r["wall_s"]) / min(r["load_s"], r["gather_s"])


def _pairs(OB, path, window, steps, n, reps, decoder=None, k=3):
    """``k`` serial / overlap runs alternated (the pool boxes' storage rate
    drifts within seconds); the pair with the median overlap/serial load
    ratio is the one checked."""
    rows = []
    for _ in range(k):
        ser = OB.run(path, window, steps, n, overlap=False, gather_reps=reps, decoder=decoder)
        ovl = OB.run(path, window, steps, n, overlap=True, gather_reps=reps, decoder=decoder)
        rows.append((ovl["load_GiBps"] / ser["load_GiBps"], ser, ovl))
    rows.sort(key=lambda r: r[0])
    print("ratios", [round(r[0], 3) for r in rows])
    return rows[len(rows) // 2][1:]


def _check(ser, ovl, steps=8):
    assert ser["verified"] and ovl["verified"]
    assert _hidden(ser) < 0.35, ser
    # the last step's side work has no next load to hide behind
    assert _hidden(ovl) >= 0.75 * (steps - 1) / steps / 0.875, (ser, ovl)
    assert ovl["wall_s"] < ser["wall_s"], (ser, ovl)
    # overlap from unslowed loads, not from loads that stretched over the side work
    assert ovl["load_GiBps"] >= 0.9 * ser["load_GiBps"], (ser, ovl)


@pytest.mark.parametrize("n", [2, 8])
def test_load_overlaps_side_stream_collective(S, tmp_path, n):
    from nvme_strom_amd.tools import overlap_bench as OB
    path = str(tmp_path / "ov.bin")
    OB._mk(path, 1 << 30)
    reps = OB.calibrate(path, 128 << 20, n)
    ser, ovl = _pairs(OB, path, 128 << 20, 8, n, reps)
    print("reps", reps, "serial", ser)
    print("overlap", ovl)
    _check(ser, ovl)


def test_load_overlaps_lds_heavy_decoder(S, tmp_path):
    """The side work is the zstd lane-parallel decoder (37-44 KB of LDS
    per entropy wave): the ingest grid, on a hardware queue of its own, keeps
    pulling loads while the decoder's workgroups hold the CUs' LDS."""
    pytest.importorskip("pyarrow")
    from nvme_strom_amd.tools import overlap_bench as OB
    path = str(tmp_path / "ovd.bin")
    OB._mk(path, 1 << 30)
    # one decode launch takes about one block's latency (~10 ms) whatever
    # its stream count: 512 MiB windows make a load the longer of the two
    dec = OB.Decoder(torch.device("cuda"), nstreams=256)
    reps = OB.calibrate(path, 512 << 20, 2, dec)
    ser, ovl = _pairs(OB, path, 512 << 20, 6, 2, reps, decoder=dec)
    print("reps", reps, "serial", ser)
    print("overlap", ovl)
    _check(ser, ovl, steps=6)

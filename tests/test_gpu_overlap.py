"""Load <-> collective overlap on one GPU.

The fan-out schedule (parallel/fanout.py) runs step i's all-gather on a side
stream while step i+1 loads through the engine's persistent ingest grid.
Here the collective is replaced by CU copy kernels on a side stream sized
like an N-rank all-gather's receive traffic (nvme_strom_amd/tools/
overlap_bench.py) and the fanout.report() overlap formula must show the
gather hidden behind the loads at N-equivalent 2 and 8."""
import os

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


@pytest.mark.parametrize("n", [2, 8])
def test_load_overlaps_side_stream_collective(S, tmp_path, n):
    from nvme_strom_amd.tools import overlap_bench as OB
    path = str(tmp_path / "ov.bin")
    OB._mk(path, 1 << 30)
    # the copy stands in for an xGMI all-gather: about half as long as a
    # load (HBM copies are far faster than xGMI, so x reps the bytes)
    reps = max(1, round(64 / (n - 1)))
    ser = OB.run(path, 128 << 20, 8, n, overlap=False, gather_reps=reps)
    ovl = OB.run(path, 128 << 20, 8, n, overlap=True, gather_reps=reps)
    print("serial", ser)
    print("overlap", ovl)
    assert ser["verified"] and ovl["verified"]
    assert ser["overlap"] is not None and ser["overlap"] < 0.35, ser
    # the last step's gather has no next load to hide behind: 7/8 at most
    assert ovl["overlap"] >= 0.75, (ser, ovl)
    assert ovl["wall_s"] < ser["wall_s"], (ser, ovl)

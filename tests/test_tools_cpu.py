"""CPU tests of the measurement tools' pure parts (no GPU)."""
import csv

from nvme_strom_amd.tools import ktrace_summary as K


def test_ktrace_summary_groups_and_rates(tmp_path, capsys):
    path = tmp_path / "tr_kernel_trace.csv"
    rows = [
        ("void (anonymous namespace)::decompress_kernel<(anonymous namespace)::Stream<4u, 2048u, 448u>,"
         " false>(int, unsigned char const*)", 0, 2000),
        ("void (anonymous namespace)::decompress_kernel<(anonymous namespace)::Stream<4u, 2048u, 448u>,"
         " false>(int, unsigned char const*)", 5000, 9000),
        ("(anonymous namespace)::crc32c_chunks_kernel(unsigned char const*, unsigned long)", 0, 250000),
        ("(anonymous namespace)::crc32c_chunks_kernel(unsigned char const*, unsigned long)", 0, 200000),
        ("(anonymous namespace)::crc32c_chunks_kernel(unsigned char const*, unsigned long)", 0, 300000),
    ]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)
    md = tmp_path / "out.md"
    assert K.main([str(path), "--bytes", "crc32c_chunks=1000000000", "--md", str(md)]) == 0
    text = md.read_text()
    # template arguments kept, parameter lists and namespaces dropped
    assert "`decompress_kernel<Stream<4u, 2048u, 448u>, false>` | 2 | 3.0 | 2.0 |" in text
    # median 250 us over 1 GB -> 4.00 TB/s
    assert "`crc32c_chunks_kernel` | 3 | 250.0 | 200.0 | 4.00 |" in text
    # the heavier kernel (total time) is listed first
    assert text.index("crc32c_chunks_kernel") < text.index("decompress_kernel")


def test_bench_shard_sizing():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    G = 1 << 30
    assert b.shard_bytes(4 * G, G, 100 * G, 0, 1) == 4 * G          # plenty of room
    assert b.shard_bytes(4 * G, G, 20 * G, 0, 8) == 2 * G           # 16 GiB over 8 ranks
    assert b.shard_bytes(4 * G, G, 20 * G, 4 * G, 8) == 2 * G       # own old shard counts
    assert b.shard_bytes(4 * G, G, 1 * G, 0, 8) == G                # never below a window
    assert b.shard_bytes(4 * G, G, int(9.9 * G), 0, 2) == 3 * G     # whole windows


def test_gpu_recipes_parse():
    """tools/gpu.sh (every committed profile's recipe) is valid bash, and the
    phases the round-6 summary cites exist in it."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "tools", "gpu.sh")
    assert subprocess.run(["bash", "-n", path]).returncode == 0
    text = open(path).read()
    for phase in ("tests", "smoke", "bench", "benchab", "probe", "lzpmc", "lppmc", "mvpmc",
                  "zatrace", "sweep", "pg", "arrow"):
        assert f"\n    {phase}) " in text, phase

"""ABI layout: the argument blocks must stay byte-compatible with nvme-strom
v0.6 (reference kmod/nvme_strom.h:17-165, measured layout in SURVEY §2.2)."""
import ctypes as C
import os
import subprocess

import pytest

from nvme_strom_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

EXPECTED_SIZES = {
    N.CheckFile: 12, N.MapGpuMemory: 32, N.UnmapGpuMemory: 8, N.ListGpuMemory: 16,
    N.InfoGpuMemory: 56, N.MemCopySsdToGpu: 72, N.MemCopyWait: 16, N.MemCopySsdToRam: 56,
    N.AllocDMABuffer: 16, N.StatInfo: 168,
    # MI355X extension (uapi.h static assertions pin the C side)
    N.MemCopySsdToGpuExtents: 80,
}

EXPECTED_OFFSETS = [
    (N.MapGpuMemory, "vaddress", 16), (N.MapGpuMemory, "length", 24),
    (N.ListGpuMemory, "handles", 8),
    (N.InfoGpuMemory, "map_offset", 32), (N.InfoGpuMemory, "paddrs", 48),
    (N.MemCopySsdToGpu, "handle", 24), (N.MemCopySsdToGpu, "offset", 32),
    (N.MemCopySsdToGpu, "file_desc", 40), (N.MemCopySsdToGpu, "chunk_ids", 56),
    (N.MemCopySsdToGpu, "wb_buffer", 64),
    (N.MemCopySsdToRam, "dest_uaddr", 24), (N.MemCopySsdToRam, "chunk_ids", 48),
    (N.StatInfo, "tsc", 8), (N.StatInfo, "nr_debug1", 104),
    (N.MemCopySsdToGpuExtents, "handle", 40), (N.MemCopySsdToGpuExtents, "extents", 72),
]


def test_extent_record_layout():
    from nvme_strom_amd.api import EXTENT_DTYPE
    assert EXTENT_DTYPE.itemsize == 24
    assert [EXTENT_DTYPE.fields[k][1] for k in ("file_off", "dst_off", "len")] == [0, 8, 16]
    assert N.MEMCPY_SSD2GPU_EXTENTS == 0x5394


@pytest.mark.parametrize("cls,size", list(EXPECTED_SIZES.items()), ids=lambda x: getattr(x, "__name__", str(x)))
def test_struct_sizes(cls, size):
    assert C.sizeof(cls) == size


@pytest.mark.parametrize("cls,field,off", EXPECTED_OFFSETS)
def test_field_offsets(cls, field, off):
    assert getattr(cls, field).offset == off


def test_ioctl_codes():
    assert N.CHECK_FILE == 0x5380
    assert N.MAP_GPU_MEMORY == 0x5381
    assert N.UNMAP_GPU_MEMORY == 0x5382
    assert N.LIST_GPU_MEMORY == 0x5383
    assert N.INFO_GPU_MEMORY == 0x5384
    assert N.ALLOC_DMA_BUFFER == 0x5385
    assert N.MEMCPY_SSD2GPU == 0x5390
    assert N.MEMCPY_SSD2RAM == 0x5391
    assert N.MEMCPY_WAIT == 0x5392
    assert N.STAT_INFO == 0x5399


def test_header_compiles_as_c_and_cxx(tmp_path):
    """The uapi header carries its own static assertions; compiling it in C
    and C++ proves the C layout equals the pinned one."""
    src = tmp_path / "probe.c"
    src.write_text('#include "strom/uapi.h"\nint main(void){return 0;}\n')
    inc = os.path.join(ROOT, "csrc", "include")
    subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-I", inc, str(src)], check=True)
    cpp = tmp_path / "probe.cc"
    cpp.write_text('#include "strom/strom.h"\nint main(){return 0;}\n')
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", inc, str(cpp)], check=True)


def test_reference_field_names_compile(tmp_path):
    """Source compatibility: code written against the v0.6 names compiles."""
    src = tmp_path / "compat.c"
    src.write_text(r'''
#include "strom/uapi.h"
int f(void) {
  StromCmd__MemCopySsdToGpu a; StromCmd__StatInfo s; StromCmd__CheckFile c;
  StromCmd__AllocDMABuffer d; StromCmd__MemCopyWait w; StromCmd__InfoGpuMemory i;
  a.nr_ram2gpu = a.nr_ssd2gpu = 0; a.wb_buffer = 0; a.relseg_sz = 0;
  s.version = 1; c.support_dma64 = 0; d.dmabuf_fdesc = -1; w.status = 0; i.paddrs[0] = 0;
  return (int)sizeof(a) + STROM_IOCTL__MEMCPY_SSD2GPU + (int)sizeof(s) + c.fdesc +
         d.node_id + (int)w.dma_task_id + (int)i.map_offset;
}
''')
    inc = os.path.join(ROOT, "csrc", "include")
    subprocess.run(["gcc", "-std=c11", "-fsyntax-only", "-I", inc, str(src)], check=True)


def test_heap_scan2_layout_matches_c(tmp_path):
    """The general heap-scan argument block (tuple descriptor + qualifier
    list) as ctypes lays it out equals the C compiler's layout."""
    src = tmp_path / "heap.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "strom/strom.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %zu %zu %zu\\n\","
        "sizeof(struct strom_heap_tupdesc), sizeof(struct strom_heap_qual),"
        "sizeof(struct strom_heap_scan2_args), offsetof(struct strom_heap_scan2_args, desc),"
        "offsetof(struct strom_heap_scan2_args, nquals), offsetof(struct strom_heap_scan2_args, quals),"
        "offsetof(struct strom_heap_scan2_args, recheck_count));return 0;}\n")
    exe = tmp_path / "heap"
    inc = os.path.join(ROOT, "csrc", "include")
    subprocess.run(["gcc", "-std=c11", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(N.HeapTupDesc), C.sizeof(N.HeapQual), C.sizeof(N.HeapScan2Args),
            N.HeapScan2Args.desc.offset, N.HeapScan2Args.nquals.offset,
            N.HeapScan2Args.quals.offset, N.HeapScan2Args.recheck_count.offset]
    assert got == want


def test_column_qual_layout_matches_c(tmp_path):
    """struct strom_col_qual / strom_qual_batch (the Arrow scan's general
    qualifier) as ops/colpred.py lays them out equals the C layout, and
    the storage/operator codes equal the header's."""
    from nvme_strom_amd.ops import colpred as CP
    src = tmp_path / "qual.c"
    src.write_text(
        '#include <stdio.h>\n#include <stddef.h>\n#include "strom/strom.h"\n'
        "int main(void){printf(\"%zu %zu %zu %zu %d %d %d %d %d %d %d %d %d\\n\","
        "sizeof(struct strom_col_qual), offsetof(struct strom_col_qual, consts),"
        "offsetof(struct strom_col_qual, offs_bytes), sizeof(struct strom_qual_batch),"
        "STROM_COL_I8, STROM_COL_U64, STROM_COL_BOOL, STROM_COL_STR32, STROM_COL_STR64,"
        "STROM_QOP_RANGES, STROM_QOP_LUT, STROM_QOP_VALID, STROM_QUAL_NAN);return 0;}\n")
    exe = tmp_path / "qual"
    inc = os.path.join(ROOT, "csrc", "include")
    subprocess.run(["gcc", "-std=c11", "-I", inc, str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(CP.ColQual), CP.ColQual.consts.offset, CP.ColQual.offs_bytes.offset,
            8 * CP.QUAL_BATCH_FIELDS, CP.COL_CODE["i1"], CP.COL_CODE["u8"], CP.COL_CODE["b1"],
            CP.COL_STR32, CP.COL_STR64, CP.QOP_RANGES, CP.QOP_LUT, CP.QOP_VALID, CP.FLAG_NAN]
    assert got == want

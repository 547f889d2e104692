// lz4par_nt512.hip — the block-parallel LZ4 decoder (lz4par.hip) with 512
// threads per stream: slices of 32 bytes, so a stream's parse, fill and
// resolve chains are half as long, at 3 resident workgroups per CU instead
// of 4 (LDS 42.9 KB; the window load unrolled 8 deep keeps it at 80 VGPRs =
// 6 waves per SIMD — 16 deep took 96 and 2 workgroups per CU).  Config-5
// frames, GB/s 512-thread vs 256-thread build (profiles/r3/dec/
// lz4par_nt_occupancy_ab.json): 512 streams 85 / 61, 768 115 / 86, 1,024
// 90 / 110, 2,048 112 / 111.  strom_decompress() takes it when a launch's
// streams fit in one round of its resident workgroups.
#define LZ4PAR_NT 512
#define LZ4P_NS lz4p512
#define LZ4PAR_ENTRY strom_decompress_par512
#define LZ4PAR_NO_HOST 1
#define LZ4PAR_LOADU 8
#define LZ4PAR_WPE_LZ4 6
// snappy too: 96 VGPRs left it at 2 workgroups per CU (5 waves per SIMD);
// at 80 (6 small spills) it keeps the third
#define LZ4PAR_WPE 6
// 32-byte slices: a 64-byte snappy run-in (512 streams val 59 -> 61, text 72 -> 74 GB/s,
// profiles/r4/dec/snappy_lookback_ab512.json)
#define LZ4PAR_SN_LOOKBACK 64
#define LZ4PAR_SN_WLOOKBACK 32
#include "lz4par.hip"

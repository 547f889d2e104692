// The block-parallel LZ4 / snappy decoder (lz4par.hip) built a third time:
// 512 threads per stream and 8 KiB output batches.  The batch's pointers
// take 33 KiB of LDS, so two workgroups fit a CU instead of three; a batch
// twice as long keeps twice the slices busy in its pointer fill (the fill
// is serial per slice, and a 4 KiB batch covers ~1/8 of a window's
// slices).  Up to two streams per CU this build wins: 512 streams, LZ4
// text / val / ids 80 / 80 / 81 -> 96 / 90 / 95 GB/s, snappy 71 / 64 / 65
// -> 91 / 78 / 81 (profiles/r4/dec/lz4par_ob8k_ab.json); at 2,048 streams
// the third resident workgroup is worth more.
#define LZ4PAR_NT 512
#define LZ4P_NS lz4p512b
#define LZ4PAR_ENTRY strom_decompress_par512b
#define LZ4PAR_NO_HOST 1
#define LZ4PAR_LOADU 8
#define LZ4PAR_OB 8192
#define LZ4PAR_WPE_LZ4 4
#define LZ4PAR_WPE 4
#define LZ4PAR_SN_LOOKBACK 64
#define LZ4PAR_SN_WLOOKBACK 32
#include "lz4par.hip"

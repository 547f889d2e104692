// lz4par_nt512.hip — the block-parallel LZ4 decoder (lz4par.hip) with 512
// threads per stream: slices of 32 bytes, so a stream's parse, fill and
// resolve chains are half as long (512 config-5 frames 61 -> 85 GB/s), at
// 2 resident workgroups per CU instead of 4 (2,048 frames 110 -> 85 GB/s:
// profiles/r3/dec/lz4par_nt_crossover.json).  strom_decompress() takes it
// when a launch's streams fit in one round of its resident workgroups.
#define LZ4PAR_NT 512
#define LZ4P_NS lz4p512
#define LZ4PAR_ENTRY strom_decompress_par512
#define LZ4PAR_NO_HOST 1
#include "lz4par.hip"

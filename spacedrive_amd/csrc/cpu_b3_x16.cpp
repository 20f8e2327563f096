// 16-lane instantiation of cpu_b3_lanes.inc (see the Makefile for its ISA flags)
#define SD_LANES 16
#define SD_CHUNKS_FN cpu_hash_chunks_x16
#define SD_PARENTS_FN cpu_hash_parents_x16
#define SD_CHUNKS_VAR_FN cpu_hash_chunks_var_x16
#include "cpu_b3_lanes.inc"

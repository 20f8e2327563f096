// 8-lane instantiation of cpu_b3_lanes.inc (see the Makefile for its ISA flags)
#define SD_LANES 8
#define SD_CHUNKS_FN cpu_hash_chunks_x8
#define SD_PARENTS_FN cpu_hash_parents_x8
#define SD_CHUNKS_VAR_FN cpu_hash_chunks_var_x8
#include "cpu_b3_lanes.inc"

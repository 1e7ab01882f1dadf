// tuning.h — the tuned constants of the gfx950 kernels, in one table.
//
// Every value was chosen by an interleaved A/B on MI355X (the profile cited
// beside it).  Kernels use them as constants: there is no alternative code
// path behind any of them.  A tuning build may override one with -D
// (hummingbird_amd/build.py build(defs=...), scripts/tune*.py); the product
// build compiles exactly these values.  Runtime tuning knobs are read only in
// tuning builds (HBEC_TUNE, kernels.h tune_knob).
#pragma once

#ifndef HBEC_TUNE
#define HBEC_TUNE 0  // 1: tune_knob() reads the environment (tuning builds only)
#endif

// ---- pipelined strided kernels (gf_apply_vec_pipe / pipe2, kernels.hip) ----
#ifndef HBEC_PIPE_BLOCK
#define HBEC_PIPE_BLOCK 256  // threads per block: 4 waves, one per SIMD
#endif
#ifndef HBEC_PIPE_BLOCKS_PER_CU
#define HBEC_PIPE_BLOCKS_PER_CU 1  // 2-3 blocks per CU: 49-64 % vs 70.75 % (profiles/r01_tune_grid.jsonl)
#endif
#ifndef HBEC_PIPE_U_BIG
#define HBEC_PIPE_U_BIG 3  // KiB per input per wave tile, 5 <= K <= 8: 8+3 74.0 % vs 72.9 % at 2 KiB
#endif
#ifndef HBEC_PIPE_SLEEP
#define HBEC_PIPE_SLEEP 6  // x 64 cycles after the next tile's loads, K <= 4 (profiles/r01_tune_sleep*.jsonl)
#endif
#ifndef HBEC_PIPE2_SLEEP
#define HBEC_PIPE2_SLEEP 8  // pipe2 with its block barrier: 6 and 8 tie, 12 loses 4 % (r01_tune_sleep_pipe2)
#endif
#ifndef HBEC_PIPE_IMAJ
#define HBEC_PIPE_IMAJ 0  // pipelined kernels: 1 = a shard's windows back to back (A/B)
#endif
#ifndef HBEC_PIPE_TEMP
#define HBEC_PIPE_TEMP 0  // pipelined kernels: 1 = input loads with the temporal hint (A/B)
#endif
#ifndef HBEC_VEC_CHUNK_TILES
// tiles per launch of the aligned strided kernels (a batch splits into
// launches of whole objects): 256 Ki tiles ran the 4096 x 1 MiB 4+2 encode
// 72.9 -> 73.8 % and reconstruct {0,1} 70.6 -> 71.5 % against 1 Mi
// (profiles/r05_ab_grid.jsonl, HBEC_CHUNK_TILES=262144); the other kernels
// keep HBEC_CHUNK_TILES' 1 Mi
#define HBEC_VEC_CHUNK_TILES 262144
#endif
#ifndef HBEC_PIPE_V2_MAXK
#define HBEC_PIPE_V2_MAXK 4  // pipe2 up to K = 4: +1.6 % at 4+2, -7 % at 8+3 (profiles/r01_tune_pipe2.jsonl)
#endif

// ---- unpipelined strided kernel (gf_apply_vec: accumulate passes) ----
#ifndef HBEC_WAVES_PER_SIMD
#define HBEC_WAVES_PER_SIMD 4  // occupancy floor
#endif
#ifndef HBEC_TILE_SMALL
#define HBEC_TILE_SMALL 4  // KiB sub-tiles per wave tile, K <= 2
#endif
#ifndef HBEC_TILE_MID
#define HBEC_TILE_MID 1  // 3 <= K <= 4
#endif
#ifndef HBEC_TILE_BIG
#define HBEC_TILE_BIG 1  // K > 4
#endif

// ---- register placement of the coefficient tables (gf_device.h) ----
#ifndef HBEC_ALLVGPR_MIN
#define HBEC_ALLVGPR_MIN 16  // K*R from which all 5 words live in VGPRs: 8+3 66 -> 73 % (SGPR spills otherwise)
#endif

// ---- packed short-shard kernels (gf_apply_packed, gf_verify_packed) ----
#ifndef HBEC_PACKED_U_BIG
#define HBEC_PACKED_U_BIG 1  // KiB per input per wave tile for K > 4: 70 % vs 57.8 % at 3 KiB
#endif
#ifndef HBEC_PACKED_MAX_BIG
#define HBEC_PACKED_MAX_BIG 32784  // 5 <= K <= 8: packed below this S (exclusive), 8+3 @ 32 KiB objects 50.5 -> 71 % (r06_ab_packed)
#endif
#ifndef HBEC_PACKED_BLOCKS_SMALL
#define HBEC_PACKED_BLOCKS_SMALL 2  // blocks per CU, K <= 4: +7-10 % over 1 (r02_tune_packed*.jsonl)
#endif
#ifndef HBEC_PACKED_BLOCKS_BIG
#define HBEC_PACKED_BLOCKS_BIG 1
#endif
#ifndef HBEC_VERIFY_PACKED_U_SMALL
#define HBEC_VERIFY_PACKED_U_SMALL 2  // 16-B elements per lane per tile, K <= 4 (r02_verify_packed_tune.jsonl)
#endif
#ifndef HBEC_VERIFY_PACKED_U_BIG
#define HBEC_VERIFY_PACKED_U_BIG 1
#endif
#ifndef HBEC_VERIFY_PACKED_BLOCKS_SMALL
#define HBEC_VERIFY_PACKED_BLOCKS_SMALL 2
#endif
#ifndef HBEC_VERIFY_PACKED_BLOCKS_BIG
#define HBEC_VERIFY_PACKED_BLOCKS_BIG 2
#endif

// ---- round-2 unaligned kernel (gf_apply_unaligned: 13..16 inputs, S > 2^31) ----
#ifndef HBEC_UNALIGNED_U
#define HBEC_UNALIGNED_U 4  // windows per wave tile: u4 > u2, 8 loses 10-20 % (r02_tune_unaligned*.jsonl)
#endif

// ---- wide kernels (gf_wide: Verify of k > 8, apply of k > 16) ----
#ifndef HBEC_WIDE_U
#define HBEC_WIDE_U 2  // windows per tile, each element's tables read once for U columns (10+4 verify 51 -> 55 %)
#endif
#ifndef HBEC_WIDE_D
#define HBEC_WIDE_D 4  // loads in flight per lane (ring depth)
#endif

// ---- odd-shard kernels (gf_odd / gf_odd_rec / gf_odd_plan, odd_impl.h) ----
#ifndef HBEC_ODD_U_SMALL
#define HBEC_ODD_U_SMALL 2  // windows per wave tile for K <= 4: 4+2 62.5 -> 65 % over 4 / K (r03_tune_odd3)
#endif
#ifndef HBEC_ODD_U_MID
#define HBEC_ODD_U_MID 1  // 5 <= K <= 8 (one window above 8); 2 / 3 windows: 8+3 encode 66.8 -> 58.8 / 55.2 % (r04_ab_odd I)
#endif
#ifndef HBEC_ODD_U_VERIFY
#define HBEC_ODD_U_VERIFY 4  // chained Verify windows per tile, K <= 4: 4+2 80.1 -> 81.3 %, traffic 1.060 -> 1.024 x (r04_ab_odd V)
#endif
#ifndef HBEC_ODD_PLAN_U
#define HBEC_ODD_PLAN_U 2  // windows per plan record: odd 4+2 stripe plan 52.9 -> 59.5 % (r03b4)
#endif
#ifndef HBEC_ODD_REC_MINKR
#define HBEC_ODD_REC_MINKR 18  // strided batches: object records (gf_odd_rec) from K R >= 18, R >= 3 above K = 8 (r04_ab_odd F, G, Q2)
#endif
#ifndef HBEC_ODD_LDS_MINK
#define HBEC_ODD_LDS_MINK 9  // record kernels: coefficient tables in LDS from K = 9 (12+4 encode 51 -> 57 %; from K = 5, 8+3 lost 5 %)
#endif
#ifndef HBEC_ODD_BP_BPC
#define HBEC_ODD_BP_BPC 1  // blocks per CU of the bit-plane apply kernels: 2 lost 5-15 points (r05_ab_bitplane r5_ab2/3)
#endif
#ifndef HBEC_ODD_BP_PF
#define HBEC_ODD_BP_PF 1  // bit-plane records issued a tile ahead where no SGPR spills (K R <= 24; off: equal, r5_ab2)
#endif
#ifndef HBEC_ODD_BP_U
#define HBEC_ODD_BP_U 2  // carried windows per bit-plane tile (column pairs); 4 lost 1-13 points (r5_ab6)
#endif
#ifndef HBEC_ODD_BP_VBARRIER
#define HBEC_ODD_BP_VBARRIER 1  // bit-plane Verify at 2 blocks per CU: one block barrier per tile (r05_ab_verify.jsonl)
#endif
// Shortest 16-B-aligned shard apply_views routes to the record kernels
// (hbec.cpp rec_route), 5 <= k <= 8 / 9 <= k <= 12: 8+3 at 32 KiB 60.8 % on
// the aligned kernel vs 56.2 %, at 64 KiB 60.6 vs 63.3 %; 10+4 at 16 KiB
// 53.8 vs 46.8 %, at 32 KiB 54.0 vs 57.1 % (r05_ab_route.jsonl, r5_route2)
#ifndef HBEC_REC_ROUTE_MIN_S
#define HBEC_REC_ROUTE_MIN_S 49152
#endif
#ifndef HBEC_REC_ROUTE_MIN_S_BIG
#define HBEC_REC_ROUTE_MIN_S_BIG 24576
#endif
#ifndef HBEC_ODD_REC_BIGK_MINKR
// 9 <= k <= 12: the record kernel (LDS tables) from K R >= 24, i.e. every
// 3-4-output pass and 12 x 2 (12+4 reconstruct {0,1} 53.3 -> 57.4 %); 9-11
// inputs x 2 outputs stay on gf_odd (10+4 reconstruct 66.2 vs 58.3 %,
// 9+3 66.8 vs 60.1 %, 10+2 66.7 vs 61.1 %; r05_ab_rr2.jsonl)
#define HBEC_ODD_REC_BIGK_MINKR 24
#endif
#ifndef HBEC_ODD_TEMP
// record-kernel input loads with the temporal hint: bit 0 Verify, bit 1 apply,
// bit 2 window-major strided apply (the 3-wave 12+4 kernel).  4: odd 12+4
// encode 61.5-62.7 -> 64.3-64.6 %, reads 1.090 -> 1.002 x; the same hint on
// its plans reads 1.071 -> 1.003 x but runs 61.0 -> 57.1 %, on 8+3 / 10+4
// apply -2.3 / -0.4, on Verify -5 to -7 points at 1.006 / 1.002 x reads
// (r05_ab_temp.jsonl, r5_temp / r5_temp2)
#define HBEC_ODD_TEMP 4
#endif
#ifndef HBEC_ODD_BP_WPB
#define HBEC_ODD_BP_WPB 4  // waves per block of the bit-plane kernels (one block per CU); 2: -7 to -12 (r5_ab5)
#endif
#ifndef HBEC_ODD_BP_WPB3_MINKR
#define HBEC_ODD_BP_WPB3_MINKR 48  // 3 waves per block from K R = 48: 12+4 58.3 -> 62.9 %, 10+4 -3 (r5_ab5/6)
#endif
#ifndef HBEC_ODD_BPC_APPLY
#define HBEC_ODD_BPC_APPLY 1  // blocks per CU of the strided / plan apply grids (register-bound shapes: odd_two_blocks)
#endif
#ifndef HBEC_ODD_BPC_VERIFY
#define HBEC_ODD_BPC_VERIFY 2  // read-only: 4+2 68.5 -> 81 % with 2 blocks per CU (r03_tune_odd3)
#endif

#ifndef HBEC_ODD_EDGE_FUSE
// apply passes that code each shard's guard-band bytes (head [0, 64), tail
// [S - 64, S)) inside the main kernel, in the shard's first / last tile,
// instead of the second gf_odd_edges launch (round 6); bit 1: gf_odd
// (K <= 4, R <= 3), bit 2: the record kernels (compiled but slower:
// odd_impl.h odd_rec_edge)
#define HBEC_ODD_EDGE_FUSE 1
#endif
#ifndef HBEC_ODD_EDGE_MAX_S
// ... for shards of at most this many bytes.  No limit: 4+2 S = 4095 47.0 ->
// 57.2-58.5 %, 6143 54.6 -> 61.2, 12287 60.7 -> 62.5, 16383 / 24575 +1.3 to
// +1.9 (one box) and -1.6 (another), 1 MiB +-0.5; 2+1 / 3+2 at S = 4095
// +10 / +13 points (r06_ab_fuse.jsonl)
#define HBEC_ODD_EDGE_MAX_S 0xFFFFFFFFull
#endif
#ifndef HBEC_ODD_EDGE_COND
// fused guard band: 1 = only a shard's first / last tile issues the K
// edge-word loads; 0 = every tile (the others from their own first column),
// so the loads in flight do not depend on the path
#define HBEC_ODD_EDGE_COND 0
#endif

// ---- ShardHash (md5.hip) ----
#ifndef HBEC_MD5_DEPTH
#define HBEC_MD5_DEPTH 2  // 64-B blocks per load group, two groups ping-ponged: 1 -> 3.85, 2 -> 2.67, 4 -> 2.79 ms
#endif
#ifndef HBEC_MD5_DEPTH_LIST
#define HBEC_MD5_DEPTH_LIST 2
#endif
// (s_setprio 3 on the chain waves beside the encode: encode + ShardHash 3.14 -> 3.39 ms, profiles/r04_md5_pipe.jsonl)
#ifndef HBEC_MD5_BLOCK
#define HBEC_MD5_BLOCK 64  // chains (lanes) per block: one wave (4-wave blocks: ShardHash alone 2.55 -> 3.45 ms, r04_md5_pipe.jsonl)
#endif

// kernels.h — launch interface of the gfx950 GF(2^8) shard kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tuning.h"

namespace hbec {

// ---- Environment knobs ----
// env_knob is the library's one reader of the environment (hbec.cpp): the
// value of `name` as an integer, dflt when unset or empty.  Operational knobs
// (the table in include/hbec.h) call it directly.  Tuning knobs call
// tune_knob, which reads the environment only in tuning builds
// (-DHBEC_TUNE=1, scripts/tune*.py); the product build compiles each to its
// default.
long long env_knob(const char* name, long long dflt);
inline long long tune_knob(const char* name, long long dflt) {
#if HBEC_TUNE
    return env_knob(name, dflt);
#else
    (void)name;
    return dflt;
#endif
}

constexpr int kMaxK = 16;         // inputs per kernel pass
constexpr uint32_t kOddListWords = 4;  // words per plan tile-list entry (PassArgs::list)
constexpr int kMaxR = 4;          // outputs per kernel pass
constexpr int kBlockThreads = 256;
constexpr int kPipeBlockThreads = HBEC_PIPE_BLOCK;  // pipelined kernel block size
constexpr int kPipeBlocksPerCu = HBEC_PIPE_BLOCKS_PER_CU;

constexpr int kVecWavesPerSimd = HBEC_WAVES_PER_SIMD;  // occupancy floor for the vec kernels

// One pass: out[r] (^)= XOR_{j<K} C[r][j] * in[j] over n_obj objects.
// Input j of object o starts at in[j] + o*in_stride[j]; likewise outputs.
struct PassArgs {
    const uint8_t* in[kMaxK];
    uint64_t in_stride[kMaxK];
    uint8_t* out[kMaxR];
    uint64_t out_stride[kMaxR];
    uint32_t tab[kMaxR][kMaxK][5];  // v_perm tables per coefficient (gf256.h perm_table)
    uint64_t n_obj;
    uint64_t shard_len;     // bytes per shard processed by this pass
    uint32_t tiles_per_obj; // vec path: ceil(shard_len / vec_tile_bytes)
    uint32_t n_tiles;       // vec path: n_obj * tiles_per_obj (< 2^32)
    uint32_t accumulate;    // 1: out ^= result (passes 2.. over >kMaxK inputs)
    uint32_t n_elems;       // packed path: n_obj * elems_per_obj (< 2^31)
    uint32_t elems_per_obj; // packed path: shard_len / 16
    uint32_t fuse;          // odd strided apply: bit 0 = code the guard band in the main kernel (HBEC_ODD_EDGE_FUSE)
    // record kernels over a plan: n_tiles entries {record index, tile in
    // record, S, edge flags} (kOddListWords u32 each; odd_rec_tile_span bytes
    // per tile); null: strided positions
    const uint32_t* list;
};

// Packed path (short shards, S < one pipelined tile, e.g. 8+3 of 4 KiB
// objects: 512 B): wave tiles run along the concatenation of every object's
// shard column, so one tile spans several objects and every lane is used.
// Kernel kinds (hbec_kernel_info): 0 unrolled, 1 pipelined, 2 streaming, 3 packed.
int is_packed_shape(int k, int r, uint64_t shard_len, int accumulate, int force_stream);
// elements (16 B) per wave tile of the packed kernel for k inputs
int packed_tile_elems(int k);
hipError_t launch_packed(int k, int r, const PassArgs& a, int grid, hipStream_t stream);
hipError_t packed_occupancy(int k, int r, int* blocks_per_cu);

// Vec path launch: fully unrolled kernel for small shapes, streaming otherwise.
int vec_tile_bytes(int k, int r, uint64_t shard_len, int accumulate, int force_stream);
int is_streaming_shape(int k, int r, int force_stream);
int is_pipe_shape(int k, int r, uint64_t shard_len, int force_stream);
// threads per block of the kernel a pass launches (pipelined vs the others)
int vec_block_threads(int k, int r, uint64_t shard_len, int accumulate, int force_stream);
// Pipelined kernels: U = 16/K KiB of each input per wave tile (K*U = 16 loads).
// Tile depth of the pipelined kernels, U KiB of each input per wave tile,
// from A/B sweeps on MI355X (profiles/r01_tune_*.jsonl): HBM streams best with
// few outstanding requests per CU — 4+2 peaks at 1 KiB tiles (4 loads per
// wave, 32 KiB in flight per CU), while 8+3 (more inputs per output byte)
// peaks at 3 KiB tiles (tuning.h).
__host__ __device__ constexpr int pipe_u(int k) { return k <= 4 ? (4 / k) : (k <= 8 ? HBEC_PIPE_U_BIG : 1); }

// Tile depth of the stripe-plan and verify kernels, from A/B runs on MI355X
// (profiles/r01_tune_plan_verify.jsonl):
//  * stripes: pipe_u for K <= 4, 1 KiB for K >= 5 — config 4's 4 KiB objects
//    (512-B shards) waste less of a shallow tile: 67.2 % vs 63.7 % at 3 KiB;
//  * verify (read-only): 4 KiB for K <= 4 (85.1 % vs 81.9 % at 1 KiB),
//    1 KiB for K >= 5 (82.0 % vs 79.8 % at 3 KiB).
__host__ __device__ constexpr int stripes_u(int k) { return k <= 4 ? pipe_u(k) : 1; }
__host__ __device__ constexpr int verify_u(int k) { return k <= 4 ? 4 : 1; }

hipError_t launch_vec(int k, int r, const PassArgs& a, int grid, hipStream_t stream, int force_stream);
// Any alignment / stride / length with aligned 16-B accesses (gf_apply_unaligned):
// wave tiles of 4 windows x 1008 B of one object's shard column.
uint32_t unaligned_tiles_per_obj(uint64_t shard_len);
hipError_t launch_unaligned(int k, int r, const PassArgs& a, int grid, hipStream_t stream);
hipError_t unaligned_occupancy(int r, int* blocks_per_cu);
// Unaligned plans (stripes / objects at any alignment, mixed lengths): one
// record per wave tile of unaligned_tile_bytes() stored bytes of a stripe.
// Input j of the tile's stripe starts at (bit j of in_sel ? b : a) +
// in_idx[j] * shard_len; output r likewise with out_sel / out_idx.
struct URec {
    uint64_t a;          // stripe base (ecSplit databuf) or object data base
    uint64_t b;          // object parity base (object plans)
    uint64_t shard_len;
    uint64_t p0;         // first window's shard position
};
struct UPlanArgs {
    const URec* recs;
    uint32_t n_recs;
    uint32_t accumulate;      // 1: out ^= result (passes beyond kMaxK inputs)
    uint32_t in_idx[kMaxK];
    uint32_t out_idx[kMaxR];
    uint32_t in_sel, out_sel;
    uint32_t tab[kMaxR][kMaxK][5];
    // gf_odd plans, zero-copy encode + ShardHash: bit 0 also stores every input
    // column, bit 1 every output column (single input pass only) to the hash
    // arena at rec.b (shard i at rec.b + i * odd_mirror_pitch_host(S))
    uint32_t mirror;
    // gf_odd plans: 1 when the records are carried 2-window tiles
    // (urec_tile_for(k, false) == 2016 B, K <= 4 passes)
    uint32_t carry;
};
uint32_t unaligned_tile_bytes();
// Verify at any alignment (k <= kMaxK, <= 4 parity rows per launch): OR 1 into
// flags[obj] for every object whose stored parity differs from the recomputed.
hipError_t launch_verify_unaligned(int k, int r, const PassArgs& a, uint32_t* flags, int grid, hipStream_t stream);
hipError_t launch_unaligned_plan(int k, int r, const UPlanArgs& a, int grid, hipStream_t stream);
// ---- odd.hip: shards at any byte offset / of any length (round 3) ----
// Aligned 16-B loads and stores only, shifted into one byte frame in
// registers (DPP lane shift + v_alignbyte); compile-time K <= kOddMaxK,
// <= kMaxR outputs; the gf_apply_vec_pipe2 schedule.  Modes: 0 apply,
// 1 accumulate (out ^= ..., later passes of k > kOddMaxK), 2 verify (flag
// objects whose stored parity differs; nothing written).
// gf_odd instances exist for K <= 8 (odd.hip, odd_k58.hip) and 9..12
// (odd_k912.hip): 10+4 odd reconstruct 51-58 -> 67 % of 8 TB/s in one pass (r3b7)
constexpr int kOddMaxK = 12;
// Longest shard the 32-bit-position kernels (gf_odd, gf_odd_plan, gf_wide)
// take.  They form shard positions in int32: column block starts, load
// limits ((l4 + S + A - 1) & ~(A - 1)) - 16, window and tile offsets, all
// below S + 4 KiB.  2^31 - 64 KiB keeps every one of them positive; longer
// shards take the 64-bit round-2 kernels (gf_apply_unaligned family).
constexpr uint64_t kPos32MaxShard = (1ull << 31) - (1ull << 16);
__host__ __device__ constexpr bool pos32_shard(uint64_t shard_len) { return shard_len <= kPos32MaxShard; }
// gf_odd for odd shards (true; a tuning build's HBEC_ODD=0 takes the round-2
// gf_apply_unaligned family instead, for A/B)
bool odd_enabled();
// 4-wave blocks per CU of a gf_odd launch (mode 0 apply, 1 accumulate, 2
// verify; K, R of the pass; records: a gf_odd_rec launch)
int odd_blocks_per_cu(int mode, int k, int r, bool mirror = false, bool records = false, int xs = -1);
bool odd_supported(int k, int r);
// Unaligned plan records (URec) of one stripe / object: p0 = 0, tile, 2*tile,
// ... while p0 < urec_span(S), for whichever kernel family codes them.
uint64_t urec_tile();
uint64_t urec_tile_for(int k, bool mirror);  // records read by a k-input pass (gf_odd carry for k <= 4)
uint64_t urec_span(uint64_t shard_len);  // 0: no main-kernel records (gf_odd: S <= odd_min_main())
uint32_t odd_tile_bytes(int k);       // shard bytes per wave tile of the strided kernel
uint32_t odd_plan_tile_bytes();       // shard bytes per plan record
// xs >= 0: the bit-plane record kernel of schedule xs (odd_bp_schedule)
uint32_t odd_tiles_per_obj(int k, int mode, uint64_t shard_len, bool records, int xs = -1);
// tiles of `tile` stored bytes per shard of shard_len > odd_min_main() bytes
uint64_t odd_frame_tiles(uint64_t shard_len, uint64_t tile);
// Bit-plane record kernels (xor_sched.h): the schedule whose fixed coefficient
// matrix equals this pass's tables (the encode parity rows of a compiled
// (k, m)) for apply (mode 0: strided or plan, XorShape strided / plan flags)
// and Verify (mode 2, strided: XorShape verify), or -1 for the v_perm table
// kernels (accumulate passes always).
int odd_bp_schedule(int k, int r, int mode, const uint32_t (*tab)[kMaxK][5], bool plan);
// shard bytes per tile of the record kernel a pass of k inputs launches (xs: odd_bp_schedule)
uint32_t odd_rec_tile_span(int k, int mode, int xs);
// waves per block of a gf_odd / gf_odd_rec launch (xs: odd_bp_schedule)
uint32_t odd_waves_per_block(int xs);
// shards of at most this many bytes are coded by gf_odd_edges alone
uint64_t odd_min_main();
// Strided passes code from per-object records (gf_odd_rec): launch_odd_objrec
// writes odd_rec_words(k, r, mode) words per object of a.n_obj objects into
// recs (device), before the main launches, whose `recs` point at their first
// object's record.  odd_uses_records(k, r): the strided kernel of that shape
// reads records (launch_odd with recs) rather than the strided bases (recs null).
bool odd_uses_records(int k, int r);
uint32_t odd_rec_words(int k, int r, int mode);
hipError_t launch_odd_objrec(int k, int r, int mode, const PassArgs& a, uint32_t* recs, hipStream_t stream);
// Plans: the same records for n stripes / objects of orecs (shard lengths
// > odd_min_main(), coded with p's shard indices and tables) into recs.
hipError_t launch_odd_planrec(int k, int r, int mode, const UPlanArgs& p, const URec* orecs, uint32_t n,
                              uint32_t* recs, hipStream_t stream);
hipError_t launch_odd(int k, int r, int mode, const PassArgs& a, uint32_t* flags, const uint32_t* recs, int grid,
                      hipStream_t stream, int xs = -1);
// a pass of this shape whose shards are at most max_s bytes codes the guard
// band inside its main kernel when PassArgs::fuse is set (HBEC_ODD_EDGE_FUSE,
// HBEC_ODD_EDGE_MAX_S: apply passes; records: the gf_odd_rec kernel, else gf_odd)
bool odd_edge_fuse(int k, int r, int mode, bool records, int xs, bool list, uint64_t max_s);
// the guard-band bytes of every shard (after the main launches of a pass;
// k <= kMaxK inputs, a.n_obj objects; verify flags mismatching objects)
hipError_t launch_odd_edges(int k, int r, int mode, const PassArgs& a, uint32_t* flags, hipStream_t stream);
// plan records: URec.p0 = first window * 992 (records cover positions [0, S + 32)),
// only for stripes longer than odd_min_main(); plus one edge record per stripe
hipError_t launch_odd_plan(int k, int r, int mode, const UPlanArgs& p, int grid, hipStream_t stream);
// lng: every record's S > kOddMinMain (the 64 + 64-slot kernel)
hipError_t launch_odd_edges_plan(int k, int r, int mode, const UPlanArgs& p, const URec* erecs, uint32_t n_erecs,
                                 hipStream_t stream, bool lng = false);
// Mirrored plans: copy shard bytes the main kernel does not mirror (the guard
// band, full = 0; whole shards, full = 1) from each edge record's stripe
// (rec.a) to its arena (rec.b), for shards idx[0 .. n_idx).
constexpr int kMirrorMaxIdx = 64;
struct MirrorCopyArgs {
    uint32_t idx[kMirrorMaxIdx];
    uint32_t n_idx;
    uint32_t full;
};
hipError_t launch_odd_mirror_copy(const URec* erecs, uint32_t n_erecs, const MirrorCopyArgs& a, hipStream_t stream);
uint64_t odd_mirror_pitch_host(uint64_t shard_len);

// ---- wide.hip: Verify of any k (k > 16 included) at any alignment, one read-only pass ----
constexpr int kWideMaxR = 8;
struct WideArgs {
    const uint64_t* in_base;    // [K] device array: input shard bases of object 0
    const uint64_t* in_stride;  // [K] object strides
    const uint32_t* tab;        // [K][wide_tab_words(R)]: coefficient (r, j) tables at j * words + 5 r
    uint64_t out[kWideMaxR];    // stored parity shard bases / strides
    uint64_t out_stride[kWideMaxR];
    uint32_t K;
    uint32_t tiles_per_obj;     // ceil(wide_main_len(S) / wide_tile_bytes())
    uint32_t n_tiles;
    uint32_t pad_;
    uint64_t shard_len;
    uint64_t n_obj;
};
uint32_t wide_tab_words(int r);
uint32_t wide_tile_bytes();
uint64_t wide_main_len(uint64_t shard_len);
// r <= kWideMaxR rows per launch; K <= 256; shard_len < 2^31.  Flags objects
// (flags[obj] |= 1) whose stored parity differs.
hipError_t launch_verify_wide(int r, const WideArgs& a, uint32_t* flags, int grid, hipStream_t stream);
// Apply of any k at any alignment in one pass (gf_wide apply + byte edges):
// outputs out[0..r) of a.n_obj objects; a.tiles_per_obj =
// wide_apply_tiles_per_obj(S) (0: the edge kernel codes every byte).
uint32_t wide_apply_tiles_per_obj(uint64_t shard_len);
hipError_t launch_apply_wide(int r, const WideArgs& a, int grid, hipStream_t stream);

// bytes (a multiple of 4) from host src to device dst, stream-ordered through
// kernel arguments (kPutWordsMax words per launch): src may go away on return
constexpr uint32_t kPutWordsMax = 960;
hipError_t launch_put_words(void* dst, const void* src, size_t bytes, hipStream_t stream);
hipError_t launch_fill(uint8_t* dst, uint64_t n_obj, uint64_t obj_len, uint64_t obj_stride, uint64_t base_seed,
                       uint64_t first, int grid, hipStream_t stream);
hipError_t vec_occupancy(int k, int r, int pipe, int force_stream, int* blocks_per_cu);

// ---- stripes (stripes.hip): mixed shard lengths in one launch ----
// One record per tile: input j of the tile starts at in_addr +
// in_idx[j]*in_stride, output r at out_addr + out_idx[r]*out_stride; lanes at
// offsets >= valid are masked on store.  In-place stripe plans use
// in_addr == out_addr and stride == shard_len; the host-path ring keeps
// inputs and outputs in separate device regions.
struct TileRec {
    uint64_t in_addr;
    uint64_t out_addr;
    uint32_t in_stride;
    uint32_t out_stride;
    uint32_t valid;
    uint32_t pad_;
};

// Stripe plans and the host ring: input j of a tile at in_addr +
// in_idx[j]*in_stride, output r at out_addr + out_idx[r]*out_stride.
// Object plans (split launches): every tile has two bases, A = (in_addr,
// in_stride) for data shards and B = (out_addr, out_stride) for parity
// shards; bit j of in_sel / out_sel picks B for input j / output r.
// At most kStripeMaxK inputs per stripes launch; more (k > 8) are split
// into passes whose later launches set `accumulate` (outputs read back).
constexpr int kStripeMaxK = 8;

struct StripeArgs {
    const TileRec* tiles;
    uint32_t n_tiles;
    uint32_t split;           // 1: object plan (in_sel / out_sel apply)
    uint32_t accumulate;      // 1: out ^= result (passes 2.. over > kStripeMaxK inputs; not with split)
    uint32_t mirror;          // 1: code in place at in_addr (stride in_stride) and copy every input and
                              //    output column to the device arena at out_addr (stride out_stride)
    uint32_t in_idx[kMaxK];   // shard index (within its base) read as input j
    uint32_t out_idx[kMaxR];  // shard index (within its base) written as output r
    uint32_t in_sel, out_sel;
    uint32_t tab[kMaxR][kMaxK][5];
};

// tile bytes of a stripes pass with k inputs; accumulate passes use 1 KiB
int stripes_tile_bytes(int k);
bool stripes_supported(int k, int r);
hipError_t launch_stripes(int k, int r, const StripeArgs& a, int grid, hipStream_t stream);
hipError_t stripes_occupancy(int k, int r, int* blocks_per_cu);

// ---- verify (verify.hip): recompute parity, compare, flag mismatching objects ----
int verify_tile_bytes(int k);
bool verify_supported(int k, int r);
hipError_t launch_verify(int k, int r, const PassArgs& a, uint32_t* flags, int grid, hipStream_t stream);
hipError_t verify_occupancy(int k, int r, int* blocks_per_cu);
hipError_t launch_compare(int r, const PassArgs& a, uint32_t* flags, int grid, hipStream_t stream);
// packed verify (short shards; same element walk as the packed apply path)
int is_verify_packed_shape(int k, int r, uint64_t shard_len);
int verify_packed_tile_elems(int k);
hipError_t verify_packed_occupancy(int k, int r, int* blocks_per_cu);
hipError_t launch_verify_packed(int k, int r, const PassArgs& a, uint32_t* flags, int grid, hipStream_t stream);

}  // namespace hbec

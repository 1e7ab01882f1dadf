// internal.h — helpers shared by the libhbec translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <exception>
#include <new>
#include <string>
#include <vector>

#include "../../include/hbec.h"
#include "kernels.h"

namespace hbec {

// Record a thread-local error message and return code.
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

// Every extern "C" entry point runs its body through this: no C++ exception
// (std::bad_alloc from a host vector, std::system_error from std::thread)
// may cross the C ABI into a Go / C caller.
template <typename F>
int guarded(const char* entry, F&& body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return fail(HBEC_ERR_NOMEM, std::string(entry) + ": host allocation failed");
    } catch (const std::exception& e) {
        return fail(HBEC_ERR_DEVICE, std::string(entry) + ": " + e.what());
    } catch (...) {
        return fail(HBEC_ERR_DEVICE, std::string(entry) + ": unknown exception");
    }
}

// Queue out[r] (^)= XOR_c coeffs[r][c] * in[c] over n_obj strided objects.
// Caps the grids of this thread's apply launches (0 = none); used around the
// encode launches of the encode + ShardHash pipeline.
void set_thread_grid_cap(int blocks);
int apply_views(int rows, int cols, const uint8_t* coeffs, const hbec_view* in, const hbec_view* out,
                uint64_t n_obj, uint64_t shard_len, hipStream_t stream);

// Stream-ordered device scratch from the library's private memory pool
// (release threshold: never), so per-call scratch costs no real allocation.
int scratch_alloc(size_t bytes, hipStream_t stream, void** out);
void scratch_free(void* p, hipStream_t stream);

// Device address of host range [p, p+len) if all of it is pinned, device-mapped
// memory (hbec_host_alloc, hipHostMalloc, hipHostRegister), else 0 (also 0 when
// HBEC_ZEROCOPY=0).  The zero-copy host paths code such memory in place.
uint64_t pinned_device_addr(const void* p, uint64_t len);
// Pinned stripes at any alignment / shard length are coded in place over PCIe
// (the gf_odd plan kernel; a tuning build's HBEC_ZC_UNALIGNED=0 stages them).
bool zero_copy_any_alignment();

// ShardHash of a list of device chains: records {addr, len, slot, 0} (32 B
// each, device memory), digest of record i at digest + slot * 16.
hipError_t launch_md5_list(const void* recs, uint64_t n, uint8_t* digest, bool aligned, hipStream_t stream);

// Per-call codec paths the coalescer (coalesce.cpp) runs for a group of one.
struct DirectFns {
    int (*encode)(hbec_codec*, uint8_t* databuf, uint64_t s);
    int (*reconstruct)(hbec_codec*, uint8_t* databuf, uint64_t s, const uint8_t* present, int data_only);
};
// Group commit of concurrent one-stripe calls (op 0 encode, 1 reconstruct)
// on databuf-layout stripes (shard i at base + i*s, n_shards = k+m).
bool coalesce_enabled();
int coalesced_call(hbec_codec* codec, int op, uint8_t* base, uint64_t s, const uint8_t* present, int n_shards,
                   int data_only, const DirectFns& fn);
void coalesce_stats(uint64_t* groups, uint64_t* calls);

// Largest shard_len hbec_encode_host_md5 accepts (a stripe must fit one
// staging slot of the host ring).
uint64_t host_md5_max_shard(const hbec_codec* codec);

// 16-B-aligned shards of k inputs that the record kernels code faster than
// the aligned ones (hbec.cpp: 9 <= k <= 12, or 5 <= k <= 8 off the 128-B
// line or with 4 rows; long enough shards); line_aligned: every base,
// stride and S % 128 == 0; bitplane: the rows have a compiled schedule
bool rec_route(int k, int rows, uint64_t shard_len, bool line_aligned, bool bitplane);
// the same for a plan of the codec's encode rows
bool plan_rec_route(const hbec_codec* c, uint64_t shard_len, bool line_aligned);

struct TileRec;
// Grid for a stripes launch of k inputs / r outputs over n_tiles records
// (one block of 4 waves per CU at most, as the strided kernels).
// blocks_per_cu > 0 overrides the HBM sweet spot (1 block per CU).
int stripes_grid(int k, int r, uint64_t n_tiles, int* grid, int blocks_per_cu = 0, int max_blocks = 0);
// out (^)= rows x in over tile records, in launches of <= 3 outputs and
// <= 8 inputs (k > 8: accumulate passes).  sel_k > 0: object-plan bases.
// mirror: code in place at each record's in_addr and copy every input and
// output column to the device arena at out_addr (StripeArgs::mirror).
// max_blocks > 0 caps the grid (zero-copy launches over PCIe).
int launch_stripe_passes(const TileRec* tiles, uint64_t n_tiles, const std::vector<int>& in_idx,
                         const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, int sel_k,
                         hipStream_t stream, int blocks_per_cu = 0, bool mirror = false, int max_blocks = 0);

struct URec;
// out (^)= rows x in over unaligned-kernel records (any alignment, mixed
// lengths), in launches of <= 4 outputs and <= kMaxK inputs (later input
// passes accumulate).  sel_k > 0: object records (indices >= sel_k are
// parity, base b).  max_blocks > 0 caps the grid (zero-copy over PCIe).
// erecs: gf_odd's one edge record per stripe (guard-band bytes; none for the round-2 kernels).
// orecs: per-stripe records of the stripes longer than odd_min_main()
// (longest s_max bytes) and their tile lists, one per record-kernel tile span
// (odd_rec_tile_span): unmirrored passes code from them (gf_odd_rec over the
// list: one launch per pass whatever the mix of lengths, no idle tiles)
// instead of recs.
struct OddTileList {
    uint32_t span = 0;            // shard bytes per tile
    const uint32_t* d = nullptr;  // device: {record index, tile in record, S, edge flags} per tile
    uint64_t n = 0;
};
constexpr int kOddSpans = 2;  // the record kernels' tile spans: 992 (5 <= K <= 12 tables), 2016 (carried 2 windows)
struct OddRecCache;  // a plan's built pass records (plan.cpp)
struct OddStripeRecs {
    OddRecCache* cache = nullptr;  // owned by the plan
    const URec* recs = nullptr;
    uint64_t n = 0, s_max = 0;
    OddTileList lists[kOddSpans];
    bool edges_long = false;  // every edge record's S > kOddMinMain (64 + 64 edge slots)
    uint64_t n_short_edges = 0;  // edge records of S <= kOddMinMain (listed first): the fused passes' edge launch
};
// the distinct odd_rec_tile_span values of apply / accumulate passes
void odd_plan_spans(uint32_t (&spans)[kOddSpans]);
int launch_unaligned_passes(const URec* recs, uint64_t n_recs, const std::vector<int>& in_idx,
                            const std::vector<int>& out_idx, const std::vector<uint8_t>& rows, int sel_k,
                            hipStream_t stream, int max_blocks = 0, const URec* erecs = nullptr,
                            uint64_t n_erecs = 0, bool mirror = false, bool round2 = false,
                            const OddStripeRecs* orecs = nullptr);

}  // namespace hbec

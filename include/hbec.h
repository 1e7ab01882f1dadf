/*
 * hbec.h — C ABI of libhbec, the MI355X (gfx950) erasure-coding engine for
 * Hummingbird's `hec` EC storage policy.
 *
 * Drop-in boundary.  In the reference the EC arithmetic is reached only
 * through github.com/klauspost/reedsolomon at six call sites in
 * objectserver/ecutils.go (:27,:59,:77,:111,:135,:168).  The plugin surface
 * above it — RegisterObjectEngine("hec", ecEngineConstructor)
 * (objectserver/ecengine.go:734-736) and the Object/ObjectStabilizer/
 * ObjectEngine interfaces (objectserver/objengine.go:35-95) — is untouched.
 * A cgo shim binds these entry points in place of the
 * klauspost Encoder (hbec_new/encode/reconstruct) and, optionally, of the
 * whole stripe loops of ecutils.go (hbec_ec_split/_reconstruct/_glue).
 *
 * Conventions: plain pointers and sizes only; 0 = success, negative = error
 * (codes map 1:1 onto the klauspost sentinels).  All entry points are
 * thread-safe (cgo calls arrive on arbitrary OS threads).  The library never
 * keeps a caller pointer after a call returns (batch calls: after the work
 * queued on the caller's stream completes).  There is NO CPU fallback inside
 * the library: a GPU failure returns HBEC_ERR_DEVICE (HBEC_ERR_NOMEM when
 * HBM or pinned host memory runs out) and the caller decides.
 */
#ifndef HBEC_H
#define HBEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Environment.  The library reads these variables once, at first use; every
 * other setting is a compiled constant (hummingbird_amd/csrc/tuning.h).
 *
 *   variable                    default  meaning
 *   HBEC_HOST_RINGS             8        host-path staging rings per device (callers beyond wait)
 *   HBEC_HOST_SLOT_MB           64       input bytes per ring slot (3 slots per ring)
 *   HBEC_HOST_THREADS           16       copy threads of a ring (capped by the host's cores;
 *                                        OMP_NUM_THREADS when set)
 *   HBEC_HASH_ARENA_MB          1024     device hash arena per ring for encode + ShardHash
 *   HBEC_ZEROCOPY               1        0: stage pinned stripes through the ring too
 *   HBEC_COALESCE               1        0: no grouping of concurrent per-call pinned calls
 *   HBEC_PERCALL_CONCURRENCY    16       per-call pageable applies at once (0: no limit)
 *   HBEC_BATCHER_WORKERS        2        batcher worker threads (1..8)
 *   HBEC_BATCHER_MD5_WORKERS    4        batcher workers for encode + ShardHash groups (0..16)
 */

/* ABI version.  2: hbec_ec_shard_length's data_shards became int64_t (Go's
 * int, as parseECScheme returns it); it was int in version 1, so a caller
 * compiled against a version-1 header must be rebuilt (a 32-bit argument
 * leaves the register's upper half undefined).  Callers may check
 * hbec_version() == HBEC_VERSION at start-up. */
#define HBEC_VERSION 2

enum {
    HBEC_OK = 0,
    HBEC_ERR_INV_SHARD_NUM = -1,   /* reedsolomon.ErrInvShardNum  (k <= 0 or m < 0)          */
    HBEC_ERR_MAX_SHARD_NUM = -2,   /* reedsolomon.ErrMaxShardNum  (k + m > 256)              */
    HBEC_ERR_TOO_FEW_SHARDS = -3,  /* reedsolomon.ErrTooFewShards                            */
    HBEC_ERR_SHARD_NO_DATA = -4,   /* reedsolomon.ErrShardNoData                             */
    HBEC_ERR_SHARD_SIZE = -5,      /* reedsolomon.ErrShardSize                               */
    HBEC_ERR_SINGULAR = -6,        /* reedsolomon errSingular (matrix.go)                    */
    HBEC_ERR_INVALID_ARG = -7,     /* bad pointer / size / flag                              */
    HBEC_ERR_DEVICE = -8,          /* HIP failure or no GPU: caller may use its own CPU codec */
    HBEC_ERR_NOMEM = -9,           /* host or device allocation failed                       */
    HBEC_ERR_UNEXPECTED_EOF = -10, /* io.ErrUnexpectedEOF (ecSplit short read)               */
    HBEC_ERR_IO = -11,             /* a reader/writer callback returned an error             */
    HBEC_ERR_SCHEME = -12          /* parseECScheme error                                    */
};

/* Human-readable name of a code; thread-local detail of this thread's last failure. */
const char* hbec_strerror(int code);
const char* hbec_last_error(void);
int hbec_version(void);

/* ---------------------------------------------------------------------------
 * Codec — replaces reedsolomon.New / Encoder (klauspost reedsolomon.go),
 * called at objectserver/ecutils.go:27,77,135.
 * ------------------------------------------------------------------------- */
typedef struct hbec_codec hbec_codec;

/* reedsolomon.New(dataShards, parityShards): builds the (k+m) x k systematic
 * matrix (Vandermonde x inv(top)).  Needs no GPU. */
int hbec_new(int data_shards, int parity_shards, hbec_codec** out);
void hbec_free(hbec_codec* codec);
int hbec_data_shards(const hbec_codec* codec);
int hbec_parity_shards(const hbec_codec* codec);
/* Copies the (k+m) x k coding matrix, row-major. */
int hbec_matrix(const hbec_codec* codec, uint8_t* out);

/* Encoder.Encode(shards) — ecutils.go:59.  shards[0..k) data, [k..k+m)
 * parity, every lens[i] equal and non-zero (else ErrShardSize /
 * ErrShardNoData); n_shards must be k+m (else ErrTooFewShards).  Parity is
 * written in place.  Host memory, synchronous. */
int hbec_encode(hbec_codec* codec, uint8_t* const* shards, const size_t* lens, int n_shards);

/* Encoder.Reconstruct (data_only = 0; ecutils.go:111) and
 * Encoder.ReconstructData (data_only = 1; ecutils.go:168).  lens[i] == 0
 * marks shard i missing; shards[i] must then point at >= S writable bytes
 * (the Go side resolves "reuse capacity or allocate").  Present shards must
 * share one length S.  On success lens[i] = S for every shard filled in. */
int hbec_reconstruct(hbec_codec* codec, uint8_t* const* shards, size_t* lens, int n_shards, int data_only);

/* Encoder.Verify (klauspost reedsolomon.go Verify): *ok = 1 when every parity
 * shard equals the parity recomputed from the data shards.  Same argument
 * checks as hbec_encode.  Host memory, synchronous. */
int hbec_verify(hbec_codec* codec, uint8_t* const* shards, const size_t* lens, int n_shards, int* ok);

/* Single-pointer forms of Encode / Reconstruct / ReconstructData / Verify
 * over ecutils.go's contiguous databuf: shard i (k+m of them) at
 * databuf + i * shard_len, exactly the slices every call site builds
 * (ecSplit ecutils.go:31-35,55-58; ecReconstruct :94-101; ecGlue :151-159).
 * A cgo caller passes &databuf[0] and scalars — no array of Go pointers, so
 * no runtime.Pinner (Go 1.10.2, the reference's toolchain, .travis.yml:7-8).
 * present: k+m bytes, non-zero = shard read (len > 0 in Go); missing shards
 * are rebuilt in their databuf slots (klauspost reuses the slice capacity,
 * which ecReconstruct/ecGlue place at the slot, ecutils.go:98-100).
 * shard_len == 0 (every shard empty) -> HBEC_ERR_SHARD_NO_DATA, as
 * klauspost's checkShards.  Host memory, synchronous. */
int hbec_encode_databuf(hbec_codec* codec, uint8_t* databuf, size_t shard_len);
int hbec_reconstruct_databuf(hbec_codec* codec, uint8_t* databuf, size_t shard_len, const uint8_t* present,
                             int data_only);
int hbec_verify_databuf(hbec_codec* codec, const uint8_t* databuf, size_t shard_len, int* ok);

/* Concurrent per-call Encode / Reconstruct / ReconstructData on databuf
 * stripes (the *_databuf entries, and hbec_encode / hbec_reconstruct when
 * the shard pointers are one buffer's consecutive slots) in pinned,
 * device-mapped memory (hbec_host_alloc) are coalesced: while at most
 * 16 such calls are inside the library each runs alone; beyond that, a call
 * that finds fewer than 2 groups in flight codes itself plus every queued
 * call of the same (device, codec, op, erasure pattern) with one zero-copy
 * launch (up to 256 MiB); a lone call runs
 * at once.  Pageable stripes run per call (their staging copies parallel on
 * the callers' threads), at most HBEC_PERCALL_CONCURRENCY (16; 0 = no limit)
 * at once, the rest waiting in arrival order.  HBEC_COALESCE=0 turns the
 * grouping off.  Counters since load: groups run and calls they carried. */
int hbec_coalesce_stats(uint64_t* groups, uint64_t* calls);

/* ---------------------------------------------------------------------------
 * Device-resident batches (the GPU hot path).  A view places shard i of
 * object o at base + o * obj_stride in device memory.  Work is queued on
 * hip_stream (a hipStream_t; NULL = default stream) and not waited for.
 * Output views must not overlap input views (as with klauspost, whose
 * outputs are separate slices): every output byte is written exactly once,
 * but a byte that is also an input of another object or column may be read
 * before or after that write.  Batches are split into launches of at most
 * 2^20 tiles of whole objects.
 * ------------------------------------------------------------------------- */
typedef struct {
    void* base;
    uint64_t obj_stride;
} hbec_view;

/* Encode n_objects objects at once: views[0..k) data, views[k..k+m) parity. */
int hbec_encode_batch(hbec_codec* codec, const hbec_view* views, uint64_t n_objects, uint64_t shard_len,
                      void* hip_stream);

/* Reconstruct with one erasure pattern for the whole batch: present[i] != 0
 * for surviving shards (read), 0 for missing ones (written).  Same row
 * selection as Encoder.Reconstruct: the first k present shards in index
 * order are the survivors.  data_only = 1 leaves missing parity untouched. */
int hbec_reconstruct_batch(hbec_codec* codec, const hbec_view* views, const uint8_t* present, uint64_t n_objects,
                           uint64_t shard_len, int data_only, void* hip_stream);

/* Verify a batch (read-only stream over k+m shards per object): sets
 * d_flags[o] (device memory, n_objects uint32, caller-zeroed) to 1 for every
 * object whose stored parity differs from the recomputed parity. */
int hbec_verify_batch(hbec_codec* codec, const hbec_view* views, uint64_t n_objects, uint64_t shard_len,
                      uint32_t* d_flags, void* hip_stream);

/* ---------------------------------------------------------------------------
 * ShardHash on the GPU.  The object server keys each stored shard by
 * hex(MD5(shard body)) (objectserver/indexdb.go:746-753) and the auditor
 * re-hashes shard files against it (objectserver/auditor.go:100-156).
 * Digests are raw 16-byte MD5s in DEVICE memory: chain (object o, view v)
 * at d_digests + (o * n_views + v) * 16 (4-byte aligned buffer).  One GPU
 * lane per chain.
 * ------------------------------------------------------------------------- */
/* MD5 of len bytes of every view of every object (len may be 0). */
int hbec_md5_batch(const hbec_view* views, int n_views, uint64_t n_objects, uint64_t len, uint8_t* d_digests,
                   void* hip_stream);

/* MD5 of n DEVICE buffers of any lengths (d_bufs and lens are host arrays):
 * digest of buffer i at d_digests + i * 16.  Chains run longest first, one
 * lane each; a launch lasts as long as its longest chain. */
int hbec_md5_list(const void* const* d_bufs, const uint64_t* lens, uint64_t n, uint8_t* d_digests,
                  void* hip_stream);

/* MD5 of n HOST buffers of any lengths — e.g. an auditor pass over shard
 * files (auditor.go:100-156) — staged through a pinned three-slot ring so the
 * gather, the H2D copies and the hashing of successive chunks overlap.
 * digests (host): buffer i at i * 16.  Synchronous. */
int hbec_md5_host(const uint8_t* const* bufs, const uint64_t* lens, uint64_t n, uint8_t* digests);

/* Streaming chains for multi-stripe shards (a shard file is the concatenation
 * of its per-stripe sub-chunks, ecutils.go:55-69): n_views x n_objects chains
 * fed any number of updates (every chain gets the same len per update), then
 * final, which also resets the context for reuse.  One thread at a time. */
typedef struct hbec_md5 hbec_md5;
int hbec_md5_new(int n_views, uint64_t n_objects, hbec_md5** out);
void hbec_md5_free(hbec_md5* ctx);
int hbec_md5_update(hbec_md5* ctx, const hbec_view* views, uint64_t len, void* hip_stream);
int hbec_md5_final(hbec_md5* ctx, uint8_t* d_digests, void* hip_stream);

/* hbec_encode_batch + the MD5 of all k+m shards of every object (digest of
 * shard i of object o at (o * (k+m) + i) * 16).  For k <= 4 the hash of
 * column segment s runs on a side stream while segment s+1 is encoded; the
 * caller's stream waits for both. */
int hbec_encode_md5_batch(hbec_codec* codec, const hbec_view* views, uint64_t n_objects, uint64_t shard_len,
                          uint8_t* d_digests, void* hip_stream);

/* The decode rows a reconstruct applies: survivors[0..k) (shard indices read),
 * outputs[0..*n_outputs) (shard indices written), rows[*n_outputs][k]. */
int hbec_decode_rows(hbec_codec* codec, const uint8_t* present, int data_only, int* survivors, int* outputs,
                     int* n_outputs, uint8_t* rows);

/* Generic GF(2^8) matrix apply on the GPU: out[r] = XOR_c coeffs[r*cols+c] * in[c]. */
int hbec_apply_batch(int rows, int cols, const uint8_t* coeffs, const hbec_view* in, const hbec_view* out,
                     uint64_t n_objects, uint64_t shard_len, void* hip_stream);

/* Synthetic objects on the GPU (bench/test inputs): object o = the
 * little-endian splitmix64 stream seeded base_seed ^ ((first+o) * 0x9E3779B97F4A7C15). */
int hbec_fill_splitmix(void* dst, uint64_t n_objects, uint64_t obj_len, uint64_t obj_stride, uint64_t base_seed,
                       uint64_t first, void* hip_stream);

/* ---------------------------------------------------------------------------
 * Stripe plans: many stripes of MIXED shard lengths in one launch.  A stripe
 * is ecSplit's databuf layout (ecutils.go:31-35,55-58): k+m shards of
 * shard_len bytes back to back at base, data first.  The plan (built
 * synchronously, device memory) records the stripes' addresses: the buffers
 * must stay allocated while work queued with the plan runs.  Stripes whose
 * base or shard_len is not 16-B aligned (most object sizes) are coded by one
 * more launch per pass of the unaligned kernel over their own records.
 * ------------------------------------------------------------------------- */
typedef struct {
    void* base;
    uint64_t shard_len;
} hbec_stripe;

typedef struct hbec_plan hbec_plan;

int hbec_plan_stripes(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes, hbec_plan** out);
/* Object plans: each object's k data shards back to back at `data` and its m
 * parity shards back to back at `parity` (two regions, e.g. a data arena and
 * a parity arena), shard_len bytes each.  Same encode / reconstruct / info /
 * free calls as stripe plans.  Keeping parity out of the data rows streams
 * faster on MI355X than ecSplit's in-row layout. */
typedef struct {
    void* data;
    void* parity;
    uint64_t shard_len;
} hbec_object;
int hbec_plan_objects(hbec_codec* codec, const hbec_object* objects, uint64_t n_objects, hbec_plan** out);
void hbec_plan_free(hbec_plan* plan);
/* n_tiles / tile_bytes: the aligned stripes' tile records; n_fallback: the
 * stripes (objects with k <= 8) coded by the any-alignment record kernels
 * instead — unaligned ones, and aligned ones those kernels code faster
 * (hbec.cpp rec_route). */
int hbec_plan_info(const hbec_plan* plan, uint64_t* n_tiles, int* tile_bytes, uint64_t* n_fallback,
                   uint64_t* shard_bytes);
/* Encode every stripe of the plan (parity shards k..k+m-1 written). */
int hbec_encode_plan(hbec_codec* codec, const hbec_plan* plan, void* hip_stream);
/* Reconstruct every stripe with one erasure pattern (as hbec_reconstruct_batch). */
int hbec_reconstruct_plan(hbec_codec* codec, const hbec_plan* plan, const uint8_t* present, int data_only,
                          void* hip_stream);

/* Host-memory batches (streaming host path): stripes in HOST memory (same
 * ecSplit layout), coded through a pinned staging ring — CPU gather, H2D,
 * kernel and D2H of successive chunks overlap on three streams.  Synchronous:
 * on return the parity (encode) or the rebuilt shards (reconstruct) are in the
 * caller's stripes.  Any k (k > 8 runs in accumulate passes).  Concurrent
 * calls share at most HBEC_HOST_RINGS (8) rings per device and wait for one
 * beyond that.  Env: HBEC_HOST_SLOT_MB (64), HBEC_HOST_THREADS.
 * Zero-copy: stripes in pinned, device-mapped host memory are coded IN PLACE
 * by the GPU over PCIe — no staging copies, no CPU gather/scatter — at any
 * alignment and shard length (unaligned ones through the unaligned kernel;
 * HBEC_ZEROCOPY=0 stages every stripe).
 * hbec_host_alloc memory qualifies on every device; memory pinned elsewhere
 * (hipHostMalloc, hipHostRegister) on the device it was pinned for.  Not for
 * hbec_encode_host_md5. */
int hbec_encode_host(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes);
/* Pinned, device-mapped, portable host memory for stripe buffers (e.g. the
 * cgo shim's databuf pool, ecutils.go:31-35), so the host path above runs
 * zero-copy on any device.  hbec_host_device_addr: the device address of
 * [p, p+len) for the calling thread's device if all of it is such memory,
 * else *dev = 0. */
int hbec_host_alloc(size_t bytes, void** out);
void hbec_host_free(void* p);
int hbec_host_device_addr(const void* p, uint64_t len, uint64_t* dev);
int hbec_reconstruct_host(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes, const uint8_t* present,
                          int data_only);
/* Several GPUs from one process (a node's object server): the stripes are
 * cut into contiguous runs of about equal bytes, one per device, coded
 * concurrently by one host thread per device (each on its own ring /
 * zero-copy path).  devices = NULL: the first n_devices visible devices
 * (n_devices <= 0: all).  Synchronous.  hbec_set_device selects the calling
 * thread's device for the device-batch and single-device host calls. */
int hbec_device_count(int* n);
int hbec_set_device(int device);
int hbec_encode_host_devices(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes, const int* devices,
                             int n_devices);
int hbec_reconstruct_host_devices(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes,
                                  const uint8_t* present, int data_only, const int* devices, int n_devices);
/* hbec_encode_host + ShardHash (indexdb.go:746-753) of every data and parity
 * shard of every stripe, computed on the GPU while the stripe is in the device
 * slot (hashing of one chunk overlaps the copies of the next): digests (host)
 * receive n_stripes * (k+m) raw MD5s, shard i of stripe s at (s*(k+m)+i)*16.
 * Every stripe must fit one staging slot (k * shard_len <= HBEC_HOST_SLOT_MB).
 * When every stripe is pinned and device-mapped (hbec_host_alloc), the stripes
 * are coded in place over PCIe and the kernel copies their shards to a device
 * hash arena as it goes (no staging copy, nothing read twice over PCIe) — at
 * any alignment and shard length (the mirrored gf_odd plan kernel when a
 * stripe is not 16-B aligned or S % 16 != 0; k > 12: the outputs are read
 * back once after the last pass).  Otherwise the
 * whole batch takes the staging ring.  hbec_host_md5_stats: calls since load
 * that took each way. */
int hbec_encode_host_md5(hbec_codec* codec, const hbec_stripe* stripes, uint64_t n_stripes, uint8_t* digests);
int hbec_host_md5_stats(uint64_t* zero_copy_calls, uint64_t* ring_calls);

/* Batching driver for concurrent callers (e.g. one cgo call per Stabilize):
 * each call submits ONE host stripe and blocks until it is coded; worker
 * threads (HBEC_BATCHER_WORKERS, default 2) each code what is queued — up to
 * max_batch_bytes / workers (max_batch_bytes 0 = 256 MiB; stripe bytes =
 * (k+m) * shard_len), or what has arrived max_wait_us after the worker
 * started waiting — with one host-path call, so up to max_batch_bytes are in
 * flight.  Requests with different ops / erasure patterns form separate
 * batches.  Any k.  The codec must outlive the batcher. */
typedef struct hbec_batcher hbec_batcher;
int hbec_batcher_new(hbec_codec* codec, uint64_t max_batch_bytes, uint32_t max_wait_us, hbec_batcher** out);
void hbec_batcher_free(hbec_batcher* batcher);
int hbec_batcher_encode(hbec_batcher* batcher, const hbec_stripe* stripe);
/* Encode + ShardHash of all k+m shards of the stripe (digests: host, (k+m)*16). */
int hbec_batcher_encode_md5(hbec_batcher* batcher, const hbec_stripe* stripe, uint8_t* digests);
int hbec_batcher_reconstruct(hbec_batcher* batcher, const hbec_stripe* stripe, const uint8_t* present, int data_only);
int hbec_batcher_stats(hbec_batcher* batcher, uint64_t* batches, uint64_t* stripes);

/* Tuning / introspection: force the runtime-K streaming kernel (0/1), and
 * report what a pass of k inputs -> r outputs over shard_len bytes of
 * 128-B-aligned, contiguous shards launches: tile bytes per wave, kind
 * (0 = unrolled, 1 = pipelined, 2 = streaming, 3 = packed, 4 = the record
 * kernel gf_odd_rec) and resident blocks per CU used to size the grid.  The
 * route to the record kernels is reported for coefficient tables; rows with
 * a compiled bit-plane schedule (8+4, 6+4 encode) may take it where this
 * reports an aligned kind (hbec.cpp rec_route). */
int hbec_set_force_stream(int on);
/* Test hook: tiles per launch of the odd-shard strided kernels (0 = the
 * default 1 Mi), so a test can make a small batch cross launch boundaries:
 * each launch rebuilds its objects' records (gf_odd_objrec) and offsets its
 * bases by its first object.  Process-wide; not for production use. */
int hbec_set_odd_chunk_tiles(uint64_t tiles);
int hbec_kernel_info(int k, int r, uint64_t shard_len, int* tile_bytes, int* kind, int* blocks_per_cu);
/* Launches since load of the odd-shard main kernels (any alignment, k <= 12
 * per pass): bitplane = the compiled XOR-network kernels of the fixed encode
 * matrices (xor_sched.h), records = the table-multiply record kernels,
 * strided = the table-multiply gf_odd / gf_odd_plan kernels.  Any pointer
 * may be NULL. */
int hbec_odd_path_stats(uint64_t* bitplane, uint64_t* records, uint64_t* strided);

/* Odd-shard guard bands (the <= 64 head and tail bytes of each shard the main
 * kernels' 16-B frame does not store): launches since load of the separate
 * guard-band kernels (gf_odd_edges / gf_odd_edges_plan), and main-kernel
 * launches that coded their guard bands themselves (the fused route, round 6).
 * Either pointer may be NULL. */
int hbec_odd_edge_stats(uint64_t* edge_launches, uint64_t* fused_launches);

/* The per-object records of strided record passes (gf_odd_rec) are kept for
 * views coded again (cached on a view set's second sighting; at most 16 sets,
 * 64 MiB).  Reports the cached sets and the calls that reused one; clear != 0
 * (a test hook: no call may be in flight on any stream) synchronises the
 * device and drops them.  Either pointer may be NULL. */
int hbec_odd_record_cache(int clear, uint64_t* entries, uint64_t* hits);

/* ---------------------------------------------------------------------------
 * ecutils.go stripe loops over io callbacks (objectserver/ecutils.go:14-186,
 * objectserver/ecobj.go:82-98, :814-824).
 * ------------------------------------------------------------------------- */
/* io.Reader.Read: returns bytes read (> 0), 0 at EOF, < 0 on error. */
typedef int64_t (*hbec_read_fn)(void* ctx, uint8_t* buf, size_t n);
/* io.Writer.Write: returns 0 when all n bytes were written, non-zero on error. */
typedef int (*hbec_write_fn)(void* ctx, const uint8_t* buf, size_t n);

/* ecShardLength (ecutils.go:14-24): ceil(length / k), 0 for length < 0.
 * data_shards is Go's int (64-bit), as parseECScheme returns it. */
int64_t hbec_ec_shard_length(int64_t length, int64_t data_shards);

/* ecSplit (ecutils.go:26-72).  writers: k+m contexts, NULL = nil writer.  A
 * failing writer is dropped for the rest of the object, as in Go. */
int hbec_ec_split(int data_shards, int parity_shards, hbec_read_fn read, void* fp, int chunk_size,
                  int64_t content_length, hbec_write_fn write, void* const* writers);

/* ecReconstruct (ecutils.go:74-132).  bodies: k+m reader contexts, NULL = nil. */
int hbec_ec_reconstruct(int data_shards, int parity_shards, hbec_read_fn read, void* const* bodies, int chunk_size,
                        int64_t content_length, hbec_write_fn write, void* const* dsts, const int* dst_chunk_num,
                        int n_dsts);

/* ecGlue (ecutils.go:134-186). */
int hbec_ec_glue(int data_shards, int parity_shards, hbec_read_fn read, void* const* bodies, int chunk_size,
                 int64_t content_length, hbec_write_fn write, void* const* dsts, int n_dsts);

/* Corrected range GET decode (opt-in; the byte-exact drop-in for CopyRange
 * is hbec_ec_copy_range below): object bytes
 * [start, end) of an object of content_length bytes.  The bodies are the k+m
 * shard streams positioned at the first shard byte of the stripe holding
 * `start` (rangeChunkAlign's shardStart, the ranged shard GETs of
 * ecobj.go:241-257); the stripes covering [start, end) are glued as ecGlue
 * does and each dst receives exactly bytes [start, end) through a
 * rangeBytesWriter (ecobj.go:826-850).  The reference passes the glue a
 * shard-byte length and a start offset modulo chunk_size rather than modulo
 * k * chunk_size (ecobj.go:238-265); this entry uses the object-byte
 * quantities, so it returns the requested bytes for every range — which
 * CHANGES the bytes on the wire compared with upstream.  Returns
 * HBEC_ERR_INVALID_ARG unless 0 <= start <= end <= content_length. */
int hbec_ec_glue_range(int data_shards, int parity_shards, hbec_read_fn read, void* const* bodies, int chunk_size,
                       int64_t content_length, int64_t start, int64_t end, hbec_write_fn write, void* const* dsts,
                       int n_dsts);

/* ecObject.CopyRange's decode, byte for byte as the reference computes it
 * (ecobj.go:238-265): shardStart, shardEnd = rangeChunkAlign(start, end,
 * chunk_size, k), shardEnd capped at content_length; the bodies (the ranged
 * shard GETs "bytes=shardStart-shardEnd") are glued as ecGlue does with
 * shardEnd - shardStart as the content length, through a rangeBytesWriter
 * {start % chunk_size, end - start}.  The reference mixes shard and object
 * units here, so for ranges that do not start in the first chunk of a stripe
 * the bytes are not object[start, end) — this entry reproduces them anyway
 * (the drop-in for ecobj.go:264-265; hbec_ec_glue_range is the corrected
 * decode).  Returns the glue's status; CopyRange itself ignores it (:264).
 * HBEC_ERR_INVALID_ARG, before any read, when start < 0 or end < start (Go
 * would panic slicing with a negative offset). */
int hbec_ec_copy_range(int data_shards, int parity_shards, hbec_read_fn read, void* const* bodies, int chunk_size,
                       int64_t content_length, int64_t start, int64_t end, hbec_write_fn write, void* const* dsts,
                       int n_dsts);

/* parseECScheme (ecobj.go:82-98): "reedsolomon/<k>/<m>/<chunk>". */
int hbec_parse_ec_scheme(const char* scheme, char* algo, size_t algo_cap, int64_t* data_shards,
                         int64_t* parity_shards, int64_t* chunk_size);

/* rangeChunkAlign (ecobj.go:814-824). */
void hbec_range_chunk_align(int64_t start, int64_t end, int64_t chunk_size, int data_shards, int64_t* out_start,
                            int64_t* out_end);

#ifdef __cplusplus
}
#endif
#endif /* HBEC_H */

/*
 * xec.h -- C ABI of the MI355X-native XOR-EC hot path (libxec_hip.so).
 *
 * This is the drop-in boundary.  It replaces the reference's GPU codec
 * functions (kenji-k6/erasure-code-benchmark, src/xorec/xorec_gpu_cmp.cuh:14-70)
 * with plain-C entry points that the reference's codec plugin layer
 * (src/algorithms/, class AbstractBenchmark, abstract_bm.hpp:18-88) can call
 * from a new XorecBenchmarkHip plugin; see INTEGRATION.md.
 *
 * Batch layout (identical to the reference, abstract_bm.cpp:4-18,
 * xorec_gpu_cmp.cu:135-144):
 *   data   : stripe c, data block i   at byte c*k*bs + i*bs
 *   parity : stripe c, parity block j at byte c*m*bs + j*bs
 *   bitmap : one byte per block, stripe c at c*(k+m): k data bytes then
 *            m parity bytes; 0 = lost, nonzero = present.
 * Parity class of data block i is i % m: parity[j] = XOR of data[i], i%m==j.
 *
 * Conventions (reference xorec_gpu_cmp.cu / xorec_gpu_cmp_bm.cpp):
 *   - the caller owns every buffer, the device bitmap scratch included; the
 *     codec allocates nothing per call;
 *   - compute calls are asynchronous on `stream` (NULL = the null stream); the
 *     caller synchronises (xorec_gpu_cmp_bm.cpp:50,67);
 *   - status codes 0..4 equal the reference XorecResult
 *     (xorec_utils.hpp:26-32); 5 and 6 are new; no exception crosses the ABI.
 *   - use before xec_init returns XEC_NOT_INITIALIZED (the reference throws,
 *     xorec_gpu_cmp.cu:39,67).
 */
#ifndef XEC_H
#define XEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;

typedef enum {
  XEC_SUCCESS = 0,           /* XorecResult::Success */
  XEC_INVALID_SIZE = 1,      /* XorecResult::InvalidSize   (bs < 256 or bs % 256) */
  XEC_INVALID_ALIGNMENT = 2, /* XorecResult::InvalidAlignment (data/parity not 64-B aligned) */
  XEC_INVALID_COUNTS = 3,    /* XorecResult::InvalidCounts (k < 1, m < 1, k % m) */
  XEC_DECODE_FAILURE = 4,    /* XorecResult::DecodeFailure (a class lost > 1 block) */
  XEC_NOT_INITIALIZED = 5,   /* new: xec_init not called / failed */
  XEC_DEVICE_ERROR = 6       /* new: a HIP runtime call or launch failed */
} xec_status;

/* Replaces xorec_gpu_init (xorec_gpu_cmp.cuh:14, .cu:7-27) and xorec_init
 * (xorec.hpp:39, xorec.cpp:16-22).  Selects `device_id` for the calling
 * thread, loads the library's kernels onto it (~10 ms once per device and
 * process, so the first codec call runs at steady-state latency) and marks
 * the library initialised.  Idempotent per device.  Unlike
 * the reference it takes no k: recovery checks are sized per call, so the
 * COMPLETE_DATA_BITMAP first-call sizing bug (xorec.cpp:16-22) cannot occur. */
xec_status xec_init(int device_id);

/* Replaces xorec_gpu_encode (xorec_gpu_cmp.cuh:28-37, .cu:29-55).
 * parity[c][j] = XOR_{i % m == j} data[c][i] for every stripe c < S.
 * Arguments are checked exactly like xorec_check_args (xorec_utils.hpp:61-86).
 * One kernel, no memset, no atomics; parity is fully overwritten.
 * The reference's num_gpu_blocks/threads_per_block launch arguments are gone:
 * the launch shape is chosen for gfx950 (see xec_set_launch). */
xec_status xec_encode(const void* d_data, void* d_parity, size_t S, size_t bs, size_t k,
                      size_t m, hipStream_t stream);

/* Replaces xorec_gpu_decode (xorec_gpu_cmp.cuh:57-68, .cu:57-115).
 * h_bitmap: S*(k+m) bytes of host memory (pinned for an asynchronous copy);
 * d_bitmap: S*(k+m) bytes of device scratch owned by the caller.
 * Host checks follow the reference: XEC_DECODE_FAILURE if ANY stripe is
 * unrecoverable (is_recoverable, xorec_utils.hpp:160-175) and then no data is
 * touched; XEC_SUCCESS without a kernel if no stripe needs recovery
 * (require_recovery, xorec_utils.hpp:144-149).  Otherwise every lost data
 * block is rebuilt:
 *   data[c][i] = parity[c][i%m] ^ XOR_{l%m == i%m, l != i} data[c][l].
 * What the kernel reads besides the batch -- a copy of h_bitmap, or the list
 * of lost data blocks the host scan found (4 bytes each; the list drives one
 * tile per lost block and 1 KiB chunk, xec_set_decode_tiling) -- is copied to
 * device buffers the library keeps, on a copy stream of its own that does not
 * wait for `stream`'s earlier work, when `stream` is busy at the call; `stream`
 * waits only for that copy before the decode kernel.  When `stream` is idle
 * (a synchronous caller) the copy goes into d_bitmap on `stream` itself, which
 * then starts at once without a cross-stream hand-off.  Up to 1,024 list
 * entries travel in the kernel arguments instead, and then nothing is copied;
 * so do batches of at most 1,024 stripes with k <= 32 that would otherwise
 * copy something (one loss mask per stripe).
 * d_bitmap is scratch for the call.  Not
 * capturable: the host scan reads h_bitmap at call time, so a graph would
 * replay this call's losses -- on a stream being captured a call with blocks
 * to rebuild returns XEC_DEVICE_ERROR with nothing queued (xec_decode_device
 * is the capturable form).  A batch that needs no recovery, or cannot be
 * recovered, returns XEC_SUCCESS / XEC_DECODE_FAILURE from the host scan
 * before any device call, capturing or not, as the reference decides before
 * its first CUDA call (xorec_gpu_cmp.cu:75-81).
 * Lost parity is not regenerated.  Parity is READ-ONLY here, as in the CPU
 * decode (xorec.cpp:62-111) -- deliberately unlike the reference GPU decode,
 * which folds all data into parity (xorec_gpu_cmp.cu:94-102).  The content of
 * lost data blocks on entry is irrelevant (no zeroing pre-condition).
 * The list is staged in pinned host memory the library keeps for reuse; the
 * pinned staging, the device buffers and one copy stream per device are the
 * only memory it holds across calls.  Bitmaps of 256 KiB and more are copied
 * before the host scan so the two overlap (into d_bitmap on the fallback path,
 * whatever the verdict).  h_bitmap must stay unchanged until the stream has
 * passed the call, as for any asynchronous copy. */
xec_status xec_decode(void* d_data, const void* d_parity, size_t S, size_t bs, size_t k,
                      size_t m, const uint8_t* h_bitmap, uint8_t* d_bitmap, hipStream_t stream);

/* Per-stripe form of xec_decode: the semantics of the reference CPU plugin
 * (XorecBenchmark::decode, xorec_bm.cpp:43-58, xorec_decode per stripe,
 * xorec.cpp:62-111) rather than of its GPU path.  Every stripe that needs
 * recovery and is recoverable is rebuilt; an unrecoverable stripe is left
 * untouched and makes the call return XEC_DECODE_FAILURE after the others
 * are queued.  h_codes (S bytes of host memory, may be NULL) receives each
 * stripe's XorecResult (0, or 4 for that stripe), written before the call
 * returns.  Always work-list tiles (one per rebuilt block and 1 KiB chunk);
 * requires k <= 256 and S <= 2^24 (else XEC_INVALID_SIZE).  Other arguments,
 * checks and the scratch as xec_decode. */
xec_status xec_decode_per_stripe(void* d_data, const void* d_parity, size_t S, size_t bs,
                                 size_t k, size_t m, const uint8_t* h_bitmap, uint8_t* d_bitmap,
                                 uint8_t* h_codes, hipStream_t stream);

/* Device-resident form of xec_decode (no reference counterpart: the reference
 * always scans a host bitmap, xorec_gpu_cmp.cu:75-83).  For callers whose
 * erasure bitmap already lives in device memory: no host scan, no copy, no
 * host synchronisation, so the call can be captured in a hipGraph.
 * Enqueues on `stream`: *d_status = 0; a check kernel that sets *d_status = 4
 * (XEC_DECODE_FAILURE) if any stripe is unrecoverable (is_recoverable,
 * xorec_utils.hpp:160-175); then the decode kernel, which does nothing if
 * *d_status != 0 (all-or-nothing, like xec_decode) and otherwise rebuilds
 * every lost data block exactly as xec_decode does.  The return value covers
 * only what the host can check (argument errors as xec_decode, d_status
 * null or not 4-B aligned -> XEC_INVALID_ALIGNMENT, d_bitmap null with S > 0
 * -> XEC_INVALID_SIZE, launch failure); nothing is queued on `stream` when an
 * argument is rejected.  The batch verdict is *d_status (device int32), valid
 * once the stream reaches it.  Tiling: stripe tiles with the single-erasure
 * residency table (no host view of the loss count), unless
 * xec_set_decode_tiling(2). */
xec_status xec_decode_device(void* d_data, const void* d_parity, size_t S, size_t bs, size_t k,
                             size_t m, const uint8_t* d_bitmap, int32_t* d_status,
                             hipStream_t stream);

/* Device-resident decode for batches where only some stripes lost blocks (no
 * reference counterpart; the device analogue of xec_decode's work-list tiles).
 * xec_decode_device launches a tile for every (stripe, 1 KiB chunk) of the
 * batch, so a batch where few stripes lost anything spends most of its
 * workgroups finding nothing to do.  Here the check kernel also lists the
 * lost data blocks into d_work (4-byte aligned device scratch of at least
 * xec_decode_device_list_bytes(S, k, m) bytes, owned by the caller), and the
 * decode is one tile per (listed block, chunk), walked by a grid fixed at
 * launch since the host never sees the count: one workgroup per 8 possible
 * tiles, between what the chip holds at once and 131,072 (xec_set_launch's
 * max_grid overrides it).  Sparse losses (1 stripe in 9): 1.7-3.9x faster
 * than xec_decode_device; losses in every stripe: 6-13 % slower, so there
 * xec_decode_device is the better call.  Everything else as xec_decode_device: no
 * host work (hipGraph-capturable), *d_status = 0 or 4 in stream order,
 * all-or-nothing, parity read-only, identical bytes.  Requires k <= 256 and
 * S <= 2^24 (else XEC_INVALID_SIZE), as does a too small work_bytes or a null
 * d_bitmap with S > 0; d_status or d_work null or not 4-B aligned ->
 * XEC_INVALID_ALIGNMENT; nothing is queued when an argument is rejected. */
xec_status xec_decode_device_list(void* d_data, const void* d_parity, size_t S, size_t bs,
                                  size_t k, size_t m, const uint8_t* d_bitmap, void* d_work,
                                  size_t work_bytes, int32_t* d_status, hipStream_t stream);

/* Scratch bytes xec_decode_device_list needs: 4 * (1 + S*m), a 4-byte count
 * and at most one 4-byte entry per parity class. */
size_t xec_decode_device_list_bytes(size_t S, size_t k, size_t m);

/* Host-only recoverability scan used by xec_decode (no GPU needed):
 * returns XEC_DECODE_FAILURE if some stripe is unrecoverable, else
 * XEC_SUCCESS and sets *needs_recovery to 1 iff some stripe needs recovery. */
xec_status xec_check_bitmap(const uint8_t* h_bitmap, size_t S, size_t k, size_t m,
                            int* needs_recovery);

/* Host-only argument check, identical to xorec_check_args
 * (xorec_utils.hpp:61-86); pointers are only tested for 64-B alignment. */
xec_status xec_check_args(const void* data, const void* parity, size_t bs, size_t k, size_t m);

/* Device-side erasure injection (the GPU analogue of
 * AbstractBenchmark::simulate_data_loss, abstract_bm.cpp:20-39, without the
 * per-block host memsets of xorec_gpu_cmp_bm.cpp:71-89): zero every block
 * whose d_bitmap byte is 0, data and parity alike. */
xec_status xec_erase(void* d_data, void* d_parity, size_t S, size_t bs, size_t k, size_t m,
                     const uint8_t* d_bitmap, hipStream_t stream);

/* Host-only erasure draw for one stripe's (k+m)-byte bitmap: the reference's
 * select_lost_blocks (src/utils/utils.cpp:100-127) with an explicit seed in
 * place of its wall clock -- `lost` draws from PCG32(RANDOM_SEED + seed,
 * stream 1) over the blocks still eligible, each draw marking its block 0 and
 * removing its parity class, so the set is always recoverable.  lost == 0
 * leaves the bitmap as it is; lost > m is XEC_INVALID_COUNTS (where the
 * reference prints and exits). */
xec_status xec_select_lost_blocks(size_t k, size_t m, size_t lost, uint8_t* h_bitmap,
                                  uint64_t seed);

/* Synthetic input generator (tests and bench): stripe c's stripe_bytes are
 * little-endian u64 splitmix64 outputs from state seed_base + c.
 * stripe_bytes % 8 == 0 and d_buf 8-B aligned, else XEC_INVALID_SIZE /
 * XEC_INVALID_ALIGNMENT. */
xec_status xec_fill_splitmix64(void* d_buf, size_t S, size_t stripe_bytes, uint64_t seed_base,
                               hipStream_t stream);

/* Device-side validation payload: the reference's
 * write_validation_pattern / validate_block (src/utils/utils.cpp:35-97) run on
 * the GPU over nblocks consecutive blocks of bs bytes.  Block b gets PCG32
 * bytes from offset 8 (state RANDOM_SEED + seed + b, stream 1 -- an explicit
 * seed instead of the reference's wall clock), its length at 4 and the
 * rotate-add checksum at 0; blocks under 16 bytes are one repeated byte.
 * xec_validate_blocks writes the number of blocks failing the check to *d_bad
 * (device memory).  16-byte alignment is required when bs % 16 == 0. */
xec_status xec_write_validation_pattern(void* d_data, size_t nblocks, size_t bs, uint64_t seed,
                                        hipStream_t stream);
xec_status xec_validate_blocks(const void* d_data, size_t nblocks, size_t bs, uint32_t* d_bad,
                               hipStream_t stream);

/* Tuning overrides: xec_set_launch, xec_set_occupancy, xec_set_decode_tiling
 * and xec_set_validate_kernel are PER THREAD -- an override applies to the
 * calls the setting thread makes afterwards and to no other thread's, so a
 * sweep on one thread cannot change the kernels another thread launches
 * concurrently (a new thread starts at the defaults).  The defaults are the
 * measured best; a plugin need not call any of them.
 *
 * Launch-shape override for tuning sweeps.  Each argument 0 = the measured default:
 *   unroll        16-byte granules per lane per class member: 1 or 2;
 *   max_grid      workgroups per launch (grid-stride beyond), 0 = one per tile;
 *   cache_policy  1 = non-temporal loads/stores (nt), 2 = default policy;
 *   block_threads workgroup size, 64 (one wave) or 256. */
xec_status xec_set_launch(int unroll, int max_grid, int cache_policy, int block_threads);

/* Residency of the encode/decode kernels (per thread, like xec_set_launch):
 * at most `waves_per_simd` (1..8; 8 = no cap) waves resident per SIMD,
 * enforced by reserving LDS per workgroup (the kernels use none).
 * 0 = automatic (the default): the cap measured fastest for the member count
 * k/m at the default launch shape -- 1 at k/m = 32, 2 at 16, 4 at 4 and 8;
 * for other member counts none below 8, 4 below 20, 2 below 56, else 1;
 * none at 1 and 2.  The reserved LDS keeps other kernels' LDS
 * users off those CUs while a launch runs.  Returns XEC_INVALID_SIZE outside
 * 0..8. */
xec_status xec_set_occupancy(int waves_per_simd);

/* Tuning / diagnostics (no reference counterpart): how xec_decode tiles the
 * batch.  0 = automatic (default): work-list tiles -- one per (lost data
 * block, 1 KiB column chunk), from the list the host scan builds -- when at
 * most 3/4 of the stripes lost a data block and the list fits the scratch
 * (k <= 256, S <= 2^24), and for lists of up to 1,024 entries wherever
 * stripe tiles would run; otherwise class tiles -- one
 * per (stripe, class, chunk), one class reduction each, encode's tiling --
 * when the batch lost more than one data block per stripe on average and at
 * least half of its S*m classes lost one, else stripe tiles -- one per
 * (stripe, chunk), rebuilding the stripe's lost blocks one after another.
 * Batches of at most 1,024 stripes with k <= 32 that would upload the bitmap
 * or a list send one loss mask per stripe in the kernel arguments instead
 * (class or stripe tiles by the same rule, nothing copied).
 * xec_decode_device (no host scan) uses stripe tiles.  1 = always stripe
 * tiles, 2 = always class tiles, 3 = work-list tiles where the list fits (else
 * the automatic bitmap choice), 4 = kernel-argument mask tiles where they
 * apply (else automatic).  Results are identical; only the speed differs.
 * XEC_INVALID_SIZE outside 0..4. */
xec_status xec_set_decode_tiling(int tiling);

/* Tuning / diagnostics (no reference counterpart): kernel shape of
 * xec_write_validation_pattern / xec_validate_blocks.  Grouped: the checksum
 * chain of a block is split across G lanes (G = its 128-byte segments past
 * the first 128 bytes, rounded up to a power of two, at most 64; 64/G blocks
 * per wave); needs bs % 128 == 0 and bs >= 256.  Lane: one lane walks a whole
 * block.  0 = automatic (default): validation grouped wherever bs allows it;
 * the pattern grouped below 2^18 blocks, lane per block from there.
 * 1 = always lane per block, 2 = grouped wherever bs allows it.  Results are
 * identical.  XEC_INVALID_SIZE outside 0..2. */
xec_status xec_set_validate_kernel(int mode);

/* Tuning (per thread, like xec_set_launch): column rotation of the encode and
 * decode tiles.  Stripe c's 1 KiB column chunk q is processed as chunk
 * (q + c*tiles) mod (chunks per block): a permutation of each block's chunks,
 * so results are identical; it changes which columns of the stripes in flight
 * together are read at once.  0 = automatic (the measured default), -1 = none,
 * 1..2^20 = that many chunks per stripe.  XEC_INVALID_SIZE outside -1..2^20. */
xec_status xec_set_rotation(int tiles);

/* The calling thread's overrides above as one value.  A caller that fans its
 * calls out to threads of its own (XorecBenchmarkHipMulti's shard workers)
 * reads them with xec_get_tuning and applies them in each worker with
 * xec_set_tuning, so every thread launches the shape the caller configured.
 * xec_set_tuning checks every field as the setters do and changes nothing
 * unless all are valid (XEC_INVALID_SIZE); a null pointer is
 * XEC_INVALID_ALIGNMENT. */
typedef struct {
  int unroll, max_grid, cache_policy, block_threads; /* xec_set_launch */
  int waves_per_simd;                                /* xec_set_occupancy */
  int decode_tiling;                                 /* xec_set_decode_tiling */
  int validate_kernel;                               /* xec_set_validate_kernel */
  int rotation;                                      /* xec_set_rotation */
} xec_tuning;
xec_status xec_get_tuning(xec_tuning* out);
xec_status xec_set_tuning(const xec_tuning* in);

/* Diagnostics: which tiling the calling thread's most recent xec_decode
 * launched -- 0 none (an error, or nothing to rebuild), then one of: */
enum {
  XEC_TILING_STRIPE = 1,   /* decode_kernel: (stripe, chunk) tiles over the bitmap */
  XEC_TILING_CLASS = 2,    /* decode_class_kernel: (stripe, class, chunk) tiles */
  XEC_TILING_LIST = 3,     /* decode_list_kernel: (lost block, chunk), list in d_bitmap */
  XEC_TILING_ARG_LIST = 4, /* decode_arglist_kernel: the same, list in the kernel arguments */
  XEC_TILING_ARG_MASK = 5, /* decode_argmask_kernel: class tiles, one loss mask per stripe
                              in the kernel arguments (S <= 1,024, k <= 32) */
  XEC_TILING_ARG_MASK_STRIPE = 6 /* the same masks over (stripe, chunk) tiles */
};
int xec_decode_tiling_used(void);
/* With XEC_TILING_ARG_LIST: how many entries the kernel-argument list of that
 * launch could hold -- 64, 256 or 1024, the smallest capacity that holds the
 * list, so a short list ships short kernel arguments; with XEC_TILING_ARG_MASK(_STRIPE)
 * the same for its S stripe masks; 0 for any other tiling. */
int xec_decode_arg_capacity_used(void);

/* Diagnostics / measurement: the calling thread's NEXT xec_encode, xec_decode,
 * xec_decode_per_stripe, xec_decode_device or xec_decode_device_list call
 * launches its encode / decode kernel with hipExtLaunchKernel and these two
 * events (either may be NULL), which the runtime records from that kernel's
 * own dispatch: hipEventElapsedTime(start, stop) is the kernel's execution
 * time, with no event packet queued between kernels (a hipEventRecord between
 * two kernels is a queue packet of its own, ~6 us of gap in the kernel trace,
 * DESIGN.md §4).  Both must be events of the stream's device created with
 * timing enabled.  The call that follows consumes the setting whether or not
 * it launches a kernel (a decode with nothing to rebuild records nothing); a
 * per-stripe decode that launches in pieces times its first piece.  The
 * pipeline calls ignore and clear it. */
xec_status xec_set_kernel_events(hipEvent_t start, hipEvent_t stop);

/* ---- host-in / host-out pipeline --------------------
 * The MI355X analogue of the reference's GPU-memory / unified-memory variants
 * (src/algorithms/xorec_gpu_ptr_bm.cpp:17-65, xorec_unified_ptr_bm.cpp:15-86,
 * src/xorec/xorec.cpp:114-320), which keep the data on the host side of the
 * link.  A pipeline owns `nstreams` (1..16) device slots of `chunk_stripes`
 * stripes on the current device; a batch in host memory is streamed through
 * them chunk by chunk: H2D -> kernel -> D2H, chunks overlapping across
 * streams.  Host buffers may be pageable (file or socket buffers) or pinned
 * (hipHostMalloc / hipHostRegister); pinned ones run at the link's rate
 * (config 3: encode 55, decode 55 GB/s of data against 57 raw), pageable ones
 * at 55 / 52.  Results bound for pageable memory go through
 * pinned bounce buffers the pipeline owns, copied out by a helper thread of
 * its own; pageable inputs are staged through two pinned buffers
 * of chunk_stripes*(k+m)*bs bytes, filled one chunk ahead by a pool of host
 * threads (4; XEC_PIPELINE_COPY_THREADS at create, 0 = none: HIP stages
 * them).  The calls return when the results are in host memory.  A
 * pipeline serves one call at a time: threads that stream concurrently each
 * create their own (the library's other entry points may be called from any
 * thread).  Each call runs on the pipeline's device and leaves the caller's
 * current device as it found it.  Same argument checks and status codes as
 * xec_encode / xec_decode. */
typedef struct xec_pipeline xec_pipeline;

xec_status xec_pipeline_create(xec_pipeline** out, size_t chunk_stripes, size_t bs, size_t k,
                               size_t m, int nstreams);
xec_status xec_pipeline_destroy(xec_pipeline* p);

/* h_data: S*k*bs bytes in, h_parity: S*m*bs bytes out. */
xec_status xec_pipeline_encode(xec_pipeline* p, const void* h_data, void* h_parity, size_t S);

/* Rebuilds lost data blocks of h_data in place from h_parity (read-only);
 * only chunks that lost a data block cross the link, and only the rebuilt
 * blocks are copied back.  All-or-nothing like xec_decode. */
xec_status xec_pipeline_decode(xec_pipeline* p, void* h_data, const void* h_parity, size_t S,
                               const uint8_t* h_bitmap);

/* Human-readable status name ("Success", "InvalidSize", ...). */
const char* xec_status_string(xec_status s);

/* Build identification, e.g. "xec-hip gfx950 <date>". */
const char* xec_build_info(void);

/* ---- node topology (diagnostics; no reference counterpart) ----------------
 * The reference drives one GPU (xorec_gpu_cmp.cu:7-16).  Config 5 scatters
 * stripe ranges from a root GPU to its peers; how those bytes travel depends
 * on the pair, so the multi-GPU runs record it:
 *   can_access_peer  hipDeviceCanAccessPeer(device, peer): 1 when `device`
 *                    can map `peer`'s memory (direct peer DMA), else 0 --
 *                    a copy between them is staged by the runtime;
 *   link_type        hipExtGetLinkTypeAndHopCount: the HSA link type
 *                    (XEC_LINK_PCIE 2, XEC_LINK_XGMI 4, ...), -1 when the
 *                    runtime reports none (device == peer, or no link);
 *   hop_count        hops of that link, -1 likewise.
 * XEC_INVALID_COUNTS for a device id outside 0..count-1, XEC_DEVICE_ERROR
 * when the runtime fails; *out is written only on success. */
enum { XEC_LINK_PCIE = 2, XEC_LINK_XGMI = 4 };
typedef struct {
  int can_access_peer;
  int link_type;
  int hop_count;
} xec_peer_link_info;
xec_status xec_peer_link(int device, int peer, xec_peer_link_info* out);

#ifdef __cplusplus
}
#endif
#endif /* XEC_H */

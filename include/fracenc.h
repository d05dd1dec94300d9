/*
 * fracenc.h — C ABI of the MI355X-native range×domain search engine.
 *
 * This is the drop-in boundary for the reference's hot path
 *   Frac2::AbstractEncodingEngine2 / CpuEncodingEngine2 → TransformEstimator2::estimate
 *   → TransformMatcher::match (sebsgit/fractencode encode/EncodingEngine2.hpp:50-112,
 *   encode/TransformEstimator2.hpp:29-48, encode/transformmatcher.h:38-111).
 * A caller owns the planes and grids; a context owns every device buffer.
 * No torch or HIP types cross this boundary: plain pointers, sizes and status ints.
 *
 * Semantics (identical to the reference on the same inputs):
 *  - domains are visited in the order given (the reference's createUniformGrid
 *    order), ties in distance go to the earliest domain and, inside a domain,
 *    to the later transform; the first candidate with distance <= rms_threshold
 *    wins (early exit); distance is the reference's unfitted fp32 error;
 *  - contrast / brightness follow TransformMatcher::match_generic bit-for-bit;
 *  - geometry: n x n ranges (n >= 2; Size32u rectangles too) and S x S domains with S > n, the pairs
 *    the reference CLI accepts (main.cpp:99); S = 2n is the decimate-then-permute path, any other
 *    pair — the CLI default 16 -> 4 (match_16to4) included — samples as RootMeanSquare does; range
 *    sides above 256 run every candidate in the reference's fp32 arithmetic (slower, same records);
 *  - results are returned in the order the ranges were given.
 * All entry points return 0 on success and a negative FRAC_E* code on error;
 * frac_last_error() gives the message.  Not thread-safe per context.
 */
#ifndef FRACENC_H
#define FRACENC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRAC_ABI_VERSION 9

/* error codes */
#define FRAC_OK 0
#define FRAC_E_INVALID (-1)     /* bad argument / geometry the engine does not support   */
#define FRAC_E_DEVICE (-2)      /* HIP runtime error                                     */
#define FRAC_E_STATE (-3)       /* call order (e.g. run before planes/grids are set)     */
#define FRAC_E_NOMEM (-4)       /* device or host allocation failed                      */

/* engines (frac_params.engine) */
#define FRAC_ENGINE_AUTO 0      /* fastest engine that supports the geometry             */
#define FRAC_ENGINE_VALU 1      /* v_dot2_u32_u16 scalar-broadcast search                */
#define FRAC_ENGINE_MFMA 2      /* f16 MFMA search with an exact integer epilogue        */
#define FRAC_ENGINE_SEA 3       /* successive elimination: exact per-candidate bound skips   */
                                /* domains that cannot win; same result, data-dependent cost */

/* flags (frac_params.flags) */
#define FRAC_FLAG_TIMING 1u     /* record per-kernel device time with HIP events         */
/* Alternative exact forms (same records, other kernels; for cross-checks, ABI 6).  They replace
 * the FRAC_MFMA_DFT / FRAC_SEA_TILED / FRAC_DECODE_UNFUSED environment knobs of ABI 5, which a
 * product build now refuses (FRAC_E_INVALID) like every other A/B knob. */
#define FRAC_FLAG_DIRECT_FORM 2u    /* MFMA engine, ratio-2 n = 8 and 16: the direct form (T GEMMs of K = n²)  */
                                    /* instead of the rotation-group Fourier form                               */
#define FRAC_FLAG_SEA_PER_RANGE 4u  /* SEA engine, n = 8, T = 4: the per-range form instead of the tiled one   */
#define FRAC_FLAG_DECODE_STEPWISE 8u /* decoder: one apply + one rms launch per iteration (no fused loop)       */

/* == Frac2::UniformGridItem (image/partition2.hpp:93-99): GridItemBase{origin, size}
 *    + GridItemData{bb_classifierBin}; 20 bytes. category -1 = not classified
 *    (recomputed on the item's own plane, as Classifier2::compare does). */
typedef struct frac_grid_item {
    uint32_t x, y, w, h;
    int32_t category;
} frac_grid_item;

/* Search parameters; the Frac::encode_parameters_t fields that reach the search
 * (encode/encode_parameters.h:5-14, encode/Encoder2.hpp:36). */
typedef struct frac_params {
    uint32_t transforms;    /* 4 = TransformMatcher::match's Id,R90,R180,R270; 8 = all of image/transform.h */
    int32_t use_classifier; /* 0 = DummyClassifier, 1 = BrightnessBlocksClassifier2 gating           */
    double rms_threshold;   /* TransformMatcher rmsThreshold (early-exit distance), default 0.0       */
    double s_max;           /* TransformMatcher sMax (|contrast| clamp when > 0), default -1.0         */
    uint32_t engine;        /* FRAC_ENGINE_*                                                           */
    uint32_t flags;         /* FRAC_FLAG_*                                                             */
} frac_params;

/* == Frac::transform_score_t (encode/datatypes.h:8-13), 32 bytes */
typedef struct frac_score {
    double distance;
    double contrast;
    double brightness;
    int32_t transform; /* Frac::TransformType */
    int32_t _pad;
} frac_score;

/* == Frac::item_match_t (encode/datatypes.h:14-19), 48 bytes */
typedef struct frac_match {
    frac_score score;
    uint32_t x, y;   /* winning domain origin */
    uint32_t sw, sh; /* winning domain size (sourceItemSize); 0,0 when no domain was eligible */
} frac_match;

/* == Frac::encode_item_t (encode/datatypes.h:20-23), 64 bytes */
typedef struct frac_encode_item {
    uint32_t x, y, w, h; /* range */
    frac_match match;
} frac_encode_item;

typedef struct frac_stats {
    uint64_t rejected_mappings; /* == TransformEstimator2::rejectedMappings() for this search   */
    uint64_t total_mappings;    /* nd * nr (Encoder2::encode_stats_t::totalMappings)              */
    uint32_t hit_ranges;        /* ranges decided by the rms threshold                           */
    uint32_t fallback_ranges;   /* ranges re-run in fp32 emulation (min error >= 2^24/16)        */
    uint32_t empty_ranges;      /* ranges with no eligible domain (default record)               */
    uint32_t engine;            /* engine that ran                                               */
    double ms_device;           /* device time of the last run (FRAC_FLAG_TIMING), else 0        */
    double ms_search;           /* device time of the search kernel alone                        */
    double ms_prep;             /* domain pool / operand build                                   */
    double ms_finish;           /* winner fit + fallback                                         */
    uint32_t search_form;       /* FRAC_FORM_*: how the search kernel computed the candidates     */
    uint32_t pad_;
    uint64_t matrix_flops;      /* MFMA flops the search issued (0 for the VALU engine)          */
    uint64_t evaluated_mappings; /* (range, domain) pairs whose error was computed: every eligible */
                                 /* pair for the exhaustive engines, the bound's survivors (SEA)   */
} frac_stats;

/* frac_stats.search_form */
#define FRAC_FORM_DOT2 0    /* VALU engine: packed-u16 v_dot2 per (range, transform, domain)       */
#define FRAC_FORM_DIRECT 1  /* MFMA engine: one f16 GEMM per transform (n²·T MACs per pair)        */
#define FRAC_FORM_FOURIER 2 /* MFMA engine, n = 8, T = 4: rotation-group Fourier form (96 MACs)    */
#define FRAC_FORM_SEA 3     /* SEA engine: bound-pruned exact evaluation (v_dot2)                */
#define FRAC_FORM_SEA_MFMA 4 /* SEA engine, n = 8, T = 4: the bound per tile pair, Fourier MFMA search */
#define FRAC_FORM_SAMPLED 5 /* range sizes outside {2,4,8,16}: per range an exact integer scan of the */
                            /* pool rows, one per (domain, transform), sampled as RootMeanSquare does  */

typedef struct frac_ctx frac_ctx;

int frac_abi_version(void);
/* The 16-hex-digit id of the sources this library was built from (compiled in by the build:
 * a hash of csrc/ and this header), "unknown" for a build that did not pass one. */
const char* frac_build_id(void);
/* FRAC_BUILD_* bits of this library build. */
#define FRAC_BUILD_TUNING 1 /* -DFRAC_TUNING: ablation variants (wrong results by design) compiled in */
int frac_build_flags(void);
/* The number of HIP devices this process sees (ABI 7), or a negative FRAC_E_DEVICE: a caller without
 * the HIP runtime (the reference's EncodingEngineCore2) registers one engine per device with it
 * (Multi-GPU). */
int frac_device_count(void);
/* NULL on failure (message via frac_last_error(NULL)). */
frac_ctx* frac_create(int device, const frac_params* params);
void frac_destroy(frac_ctx* ctx);
const char* frac_last_error(const frac_ctx* ctx);
int frac_set_params(frac_ctx* ctx, const frac_params* params);

/* Planes are uint8, row-major with the given stride (bytes). Copied to the device.
 * frac_set_frame: source == target (what Encoder2 does, encode/Encoder2.hpp:36).
 * frac_set_planes: distinct source (domain) and target (range) planes, as
 * TransformEstimator2's constructor allows (encode/TransformEstimator2.hpp:15-21). */
int frac_set_frame(frac_ctx* ctx, const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride);
int frac_set_planes(frac_ctx* ctx, const uint8_t* src, uint32_t sw, uint32_t sh, uint32_t sstride,
                    const uint8_t* tgt, uint32_t tw, uint32_t th, uint32_t tstride);
/* Planes already in device memory (e.g. a torch tensor in HBM): copied device-to-device. */
int frac_set_frame_device(frac_ctx* ctx, const void* d_plane, uint32_t w, uint32_t h, uint32_t stride);
/* ABI 9: the same copy enqueued on the context's stream without waiting for it, so a caller can stream
 * frames: upload frame k+1 on a stream of its own while frame k searches, make the context's stream wait
 * for that upload (an event), then call this and frac_run.  d_plane must stay unchanged until the
 * context's stream has passed the copy (an event recorded on it after this call).  The first frame of a
 * geometry, or any frame with the classifier on, re-prepares on the host in the next frac_run. */
int frac_set_frame_device_async(frac_ctx* ctx, const void* d_plane, uint32_t w, uint32_t h, uint32_t stride);
/* ABI 9: frame streaming from host memory.  The plane (pinned host memory for an asynchronous copy) is uploaded
 * on the context's own copy stream into a second plane buffer while the runs already enqueued still read the
 * current one; the context's stream waits for the upload and the buffers swap.  frac_run right after it
 * searches the new frame, so frame k+1 crosses PCIe while frame k searches.  The host plane must stay unchanged
 * until the upload is done: until a later frac_sync / frac_fetch, or an event recorded on the context's stream
 * after this call. */
int frac_set_frame_async(frac_ctx* ctx, const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride);

/* The domain pool (TransformEstimator2's sourceGrid) and the range list. */
int frac_set_domains(frac_ctx* ctx, const frac_grid_item* domains, size_t nd);
int frac_set_ranges(frac_ctx* ctx, const frac_grid_item* ranges, size_t nr);

/* Launch the whole search for the current planes/grids on the context's stream
 * (asynchronous).  frac_fetch waits for it and copies results/stats to the host. */
int frac_run(frac_ctx* ctx);
int frac_fetch(frac_ctx* ctx, frac_encode_item* out, frac_stats* stats);
int frac_sync(frac_ctx* ctx);

/* Per-run device times (FRAC_FLAG_TIMING): the ms_device / ms_prep / ms_search / ms_finish of
 * every frac_run since the previous call that passed `out` (at most the last 256 runs), oldest
 * first, from HIP events recorded on the context's stream around each phase.  Waits for the
 * stream.  *n_out = the run count; writes min(count, cap) entries (out may be NULL to query).
 * Lets a benchmark time the search kernel of exactly the runs of its timed region. */
typedef struct frac_run_timing {
    double ms_device, ms_prep, ms_search, ms_finish;
} frac_run_timing;
int frac_timing_history(frac_ctx* ctx, frac_run_timing* out, size_t cap, size_t* n_out);

/* One-shot: set_ranges + run + fetch (the shape of AbstractEncodingEngine2::encode
 * applied to a batch of range items). */
int frac_search(frac_ctx* ctx, const frac_grid_item* ranges, size_t nr, frac_encode_item* out, frac_stats* stats);

/* Use an external hipStream_t (passed as void*); NULL restores the context's own.  Work the context
 * enqueued on its previous stream comes before anything it enqueues on the new one (an event). */
int frac_set_stream(frac_ctx* ctx, void* hip_stream);
void* frac_get_stream(frac_ctx* ctx);
/* Device pointer to the nr frac_encode_item results of the last run (valid until
 * the next set_ranges / destroy); used for device-side gathers (RCCL). */
const frac_encode_item* frac_device_results(frac_ctx* ctx);
/* Asynchronous device-to-device copy of the last run's nr results into d_dst
 * (ordered on the context's stream). */
int frac_copy_results_device(frac_ctx* ctx, void* d_dst);

/* The winner of one range as north_star's multi-GPU gather names it — (domain, transform,
 * s, o, rms) — in 32 bytes instead of the 64-byte encode_item_t: the range geometry is
 * known to every rank and the domain's origin and size follow from its index.
 * domain = index into the list given to frac_set_domains; FRAC_NO_DOMAIN when no domain
 * was eligible (the default record of encode/datatypes.h:8-26). */
#define FRAC_NO_DOMAIN 0xffffffffu
typedef struct frac_tuple {
    uint32_t domain;
    int32_t transform;
    double contrast, brightness, distance;
} frac_tuple;
/* Asynchronous: pack the last run's nr tuples into d_dst (device memory, 32·nr bytes) on
 * the context's stream. */
int frac_copy_tuples_device(frac_ctx* ctx, void* d_dst);
/* Synchronous: the last run's nr tuples into host memory. */
int frac_fetch_tuples(frac_ctx* ctx, frac_tuple* out);
/* ABI 8: every later frac_run also writes its nr tuples into dst (32·nr bytes; device memory, or pinned host
 * memory the device can write — then they cross PCIe while the run's resolve kernels write them, with no
 * separate pack or copy), ordered on the context's stream: complete once that stream's work is.  The records
 * (frac_fetch, …) are unchanged.  NULL clears it.  The quadtree entry points ignore it. */
int frac_set_tuple_sink(frac_ctx* ctx, void* dst);

/* Decoder2::decode (encode/Encoder2.hpp:67-99) on the device.  `plane` (w×h, row
 * stride w) holds the decoder's initial target (main.cpp:171-173 zero-fills it) and
 * receives the decoded image; the source starts filled with 100.  Items must not
 * overlap; items without a domain (size 0) are skipped.  max_iter < 0 means 300.
 * Writes the iteration count and the final rms exactly as Decoder2 reports them. */
int frac_decode(frac_ctx* ctx, const frac_encode_item* items, size_t n, uint32_t w, uint32_t h, int max_iter,
                double rms_eps, uint8_t* plane, int* iterations, double* rms);
/* The same for the last frac_run's results, which stay on the device. */
int frac_decode_results(frac_ctx* ctx, uint32_t w, uint32_t h, int max_iter, double rms_eps, uint8_t* plane,
                        int* iterations, double* rms);

/* ---- quadtree partition (C4 config; the reference parses --quadtree but never builds one,
 * main.cpp:75-76, so the partition rule is this library's, parity pinned per level) ----
 * Level sizes max_size, max_size/2, ..., min_size (each 2, 4, 8 or 16).  Level-0 ranges are
 * createUniformGrid(W, H, max_size, max_size); every level searches domains
 * createUniformGrid(W, H, 2n, n) of the frame set on ctx (classifier and threshold as in the
 * ctx params; -1 categories are computed on the device).  A range whose best distance exceeds
 * split_distance and whose size exceeds min_size is replaced by its four quadrants (top-left,
 * top-right, bottom-left, bottom-right) at the next level; every other range is emitted.
 * Output order: by level, then in search order (children follow their parent's order).
 * Returns FRAC_OK and the item count in *n_out; writes min(count, cap) items (out may be NULL
 * to query the count — the search still runs).  stats (optional) sums the levels. */
typedef struct frac_quadtree_params {
    uint32_t max_size;
    uint32_t min_size;
    double split_distance;
} frac_quadtree_params;
int frac_encode_quadtree(frac_ctx* ctx, const frac_quadtree_params* qp, frac_encode_item* out, size_t cap,
                         size_t* n_out, frac_stats* stats);
/* The same partition with each leaf in 32 bytes instead of encode_item_t's 64 (ABI 7): what the frame's
 * geometry does not already determine.  A leaf of level size n at (x, y) won domain `code & 0xffffff` of
 * that level's grid createUniformGrid(W, H, 2n, n) — origin ((d % cols)·n, (d / cols)·n) with
 * cols = (W − 2n)/n + 1, size 2n — under transform (code >> 24) & 15; n = 1 << (code >> 28).
 * FRAC_QT_NO_DOMAIN: no eligible domain (the reference's default record: domain (0, 0), size (0, 0)).
 * The doubles are the record's own, bit for bit.  Frames up to 65535 pixels a side whose finest level
 * has fewer than 2^24 − 1 domains.  Into the caller's pinned host memory the device writes them directly,
 * half the PCIe bytes of the 64-byte records. */
#define FRAC_QT_NO_DOMAIN 0xffffffu
typedef struct frac_qt_leaf {
    uint16_t x, y;  /* range origin */
    uint32_t code;  /* domain index (bits 0..23) | transform (24..27) | log2 n (28..31) */
    double contrast, brightness, distance;
} frac_qt_leaf;
int frac_encode_quadtree_leaves(frac_ctx* ctx, const frac_quadtree_params* qp, frac_qt_leaf* out, size_t cap,
                                size_t* n_out, frac_stats* stats);

/* ---- classifier pre-pass on the device (BrightnessBlocksClassifier2::preclassify,
 * encode/Classifier2.cpp:55-68, as main.cpp:155-162 runs it at grid build) ----
 * Writes the category (0..5 or -1) of each item, computed on the context's source plane
 * (target_plane = 0) or target plane (1) already on the device.  frac_run does the same
 * internally for any item whose stored category is -1 when use_classifier is set. */
int frac_classify_items(frac_ctx* ctx, frac_grid_item* items, size_t n, int target_plane);

/* ---- frame loader: colour conversion (ImageIO::rgb2yuv, image/ImageIO.cpp:43-58) ----
 * Packed RGB (w×h, rgb_stride bytes per row) → Y (w×h) and U, V (w/2 × h/2, the odd
 * pixel of each 2×2 quad), bit-exact with the built reference (FMA-contracted weights).
 * Replaces the conversion inside ImageIO::loadImage (ImageIO.cpp:60-66); the PNG decode
 * itself stays on the host.  _device: all pointers are device pointers, the work is
 * enqueued on the ctx stream (call frac_sync before reading).  The host variant uploads,
 * converts on the device and downloads. */
int frac_rgb_to_yuv_device(frac_ctx* ctx, const void* d_rgb, uint32_t w, uint32_t h, uint32_t rgb_stride, void* d_y,
                           uint32_t y_stride, void* d_u, uint32_t u_stride, void* d_v, uint32_t v_stride);
int frac_rgb_to_yuv(frac_ctx* ctx, const uint8_t* rgb, uint32_t w, uint32_t h, uint32_t rgb_stride, uint8_t* y,
                    uint8_t* u, uint8_t* v);

/* ---- FRC1 quantized stream, packed on the device --------------------------
 * The reference has no file format; encode_data_statistics (main.cpp:106-140) builds
 * Frac::Quantizerd over the frame's (contrast, brightness) range with 5 / 7 bits
 * (main.cpp:120-121).  FRC1 (fractencode_amd/codec.py documents the layout) stores per
 * range (domain index, transform, q_contrast, q_brightness) bit-packed after a 72-byte
 * header.  This packs the last run's results into it: min/max reductions, Quantizer codes
 * (encode/Quantizer.hpp:7-45, FP64 as the reference) and the bit packing all run on the
 * device; only the finished stream is copied out.  Requires the ranges to be the
 * createUniformGrid(range_size, range_size) lattice in row-major order and the domains the
 * createUniformGrid(2·range_size, range_size) lattice (the CLI's grids, main.cpp:147-152).
 * contrast_bits, brightness_bits in [2, 16].  *n_out = stream size; writes min(cap, size)
 * bytes (out may be NULL to query the size). */
#define FRAC_FRC1_HEADER_BYTES 72
int frac_pack_frc1(frac_ctx* ctx, uint32_t contrast_bits, uint32_t brightness_bits, uint8_t* out, size_t cap,
                   size_t* n_out);

/* ---- host helpers (no device needed) ------------------------------------ */
/* createUniformGrid (image/partition2.hpp:109-135): returns the item count and
 * writes min(count, cap) items (categories -1).  Returns 0 where the reference's loop has no
 * meaningful grid: a zero size or offset (it never ends) or an item larger than the plane (its
 * do-while emits one item outside the plane, which every search entry refuses). */
size_t frac_uniform_grid(uint32_t width, uint32_t height, uint32_t item_size, uint32_t item_offset,
                         frac_grid_item* out, size_t cap);
/* The same with createUniformGrid's Size32u item size and offset (partition2.hpp:110-113): items
 * size_w × size_h, x stepping by off_x, rows by off_y (e.g. tests/OpenCLTest.cpp:76-78's 4×4 items
 * at offset (4, 2)). */
size_t frac_uniform_grid2(uint32_t width, uint32_t height, uint32_t size_w, uint32_t size_h, uint32_t off_x,
                          uint32_t off_y, frac_grid_item* out, size_t cap);
/* BrightnessBlocksClassifier2::preclassify over items (encode/Classifier2.cpp:64-68):
 * writes each item's category computed on `plane`. */
int frac_classify(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride, frac_grid_item* items, size_t n);
/* The ratio-2 sample permutation the kernels use: range pixel pix = y·n + x under
 * transform t meets decimated domain cell frac_transform_index(n, t, pix)
 * (image/sampler.h:21-38 with image/transform.h:96-109).  −1 on bad arguments. */
int frac_transform_index(uint32_t n, uint32_t t, uint32_t pix);
/* Largest integer S16 = 16·Σ(r − d̄)² whose reference distance (S16/16)/(4n²) is
 * <= rms_threshold, or −1 (TransformMatcher::checkDistance, transformmatcher.h:32-34). */
int64_t frac_hit_limit(double rms_threshold, uint32_t n);

#ifdef __cplusplus
}
#endif

#endif /* FRACENC_H */

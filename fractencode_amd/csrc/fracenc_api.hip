// fracenc_api.hip — C ABI (include/fracenc.h): contexts, host-side bucketing of the
// domain pool by classifier category, work lists, kernel launches and statistics.
//
// Host logic mirrored from the reference:
//   classifier gating      encode/Classifier2.cpp:8-81   (categories computed on the host,
//                          a stored −1 re-computed on the item's own plane like compare())
//   rejected-mapping count encode/TransformEstimator2.hpp:43-45,59 (derived from the winner)
//   search order / ties    encode/TransformEstimator2.hpp:29-48
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fracenc_common.h"
#include "fracenc_kernels.hip"
#include "fracenc_mfma.hip"
#include "fracenc_dft.hip"
#include "fracenc_decode.hip"
#include "fracenc_color.hip"
#include "fracenc_classify.hip"
#include "fracenc_sea.hip"
#include "fracenc_stream.hip"
#include "fracenc_tp.hip"
#include "fracenc_gen.hip"
#include "fracenc_bucket.hip"

using namespace fracenc;

namespace {

thread_local std::string g_last_error;

// (key, value) radix sort of u32 pairs on the low `bits` key bits. rocPRIM's default picks a
// block-sort + merge-sort path below 2^20 items: 17 launches for the 2^18 keys of a C3 frame,
// whose launch gaps cost more than the sort. Merge-sort limit 0 selects Onesweep (histogram +
// one pass per 8-bit digit).
using OnesweepConfig =
    rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
hipError_t sort_pairs_u32(void* tmp, size_t& bytes, const uint32_t* kin, uint32_t* kout, const uint32_t* vin,
                          uint32_t* vout, uint32_t n, uint32_t bits, hipStream_t s)
{
    return rocprim::radix_sort_pairs<OnesweepConfig>(tmp, bytes, kin, kout, vin, vout, n, 0u, bits, s);
}

template <class T>
struct DBuf {
    T* ptr = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n)
    {
        if (n <= cap && ptr)
            return hipSuccess;
        if (ptr)
            (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(n, 1);
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&ptr), want * sizeof(T));
        if (e == hipSuccess)
            cap = want;
        return e;
    }
    void release()
    {
        if (ptr)
            (void)hipFree(ptr);
        ptr = nullptr;
        cap = 0;
    }
};

struct HostPlane {
    std::vector<uint8_t> data; // tightly packed, stride == w
    uint32_t w = 0, h = 0;
};

// --- classifier (host) -------------------------------------------------------
// ImageStatistics2::sum (image/ImageStatistics.hpp:12-17): u16 up to 16 wide.
double block_sum(const HostPlane& p, uint32_t x, uint32_t y, uint32_t w, uint32_t h)
{
    uint32_t s = 0;
    for (uint32_t j = 0; j < h; ++j) {
        const uint8_t* row = p.data.data() + (size_t)(y + j) * p.w + x;
        for (uint32_t i = 0; i < w; ++i)
            s += row[i];
    }
    return w <= 16 ? (double)(uint16_t)s : (double)s;
}

// BrightnessBlocksClassifier2::getCategory(a1..a4) — encode/Classifier2.cpp:8-62
int category4(double a1, double a2, double a3, double a4)
{
    // rule (i, j, k): a_i > a_j && a_j > a_k && a_k > a_l, listed as quadruples (i j k l)
    static const unsigned char rules[24][4] = {
        {1, 2, 3, 4}, {3, 1, 4, 2}, {4, 3, 2, 1}, {2, 4, 1, 3}, // 0
        {1, 3, 2, 4}, {2, 1, 4, 3}, {4, 2, 3, 1}, {3, 4, 1, 2}, // 1
        {1, 4, 3, 2}, {4, 1, 2, 3}, {3, 2, 4, 1}, {2, 3, 1, 4}, // 2
        {1, 2, 4, 3}, {3, 1, 2, 4}, {4, 3, 1, 2}, {2, 4, 3, 1}, // 3
        {2, 1, 3, 4}, {1, 3, 4, 2}, {3, 4, 2, 1}, {4, 2, 1, 3}, // 4
        {1, 4, 2, 3}, {4, 1, 3, 4}, {2, 3, 4, 1}, {3, 2, 1, 4}, // 5
    };
    const double a[5] = {0.0, a1, a2, a3, a4};
    for (int r = 0; r < 24; ++r) {
        const unsigned char* q = rules[r];
        if (a[q[0]] > a[q[1]] && a[q[1]] > a[q[2]] && a[q[2]] > a[q[3]])
            return r / 4;
    }
    return -1;
}

int category(const HostPlane& p, const frac_grid_item& it)
{
    const uint32_t hw = it.w / 2, hh = it.h / 2;
    return category4(block_sum(p, it.x, it.y, hw, hh), block_sum(p, it.x + hw, it.y, hw, hh),
                     block_sum(p, it.x, it.y + hh, hw, hh), block_sum(p, it.x + hw, it.y + hh, hw, hh));
}

// Largest S16 whose reference distance fl64((S16/16)/area) is <= thr
// (TransformMatcher::checkDistance, encode/transformmatcher.h:32-34); −1 if none.
int64_t compute_hit_limit(double thr, uint32_t area)
{
    auto pred = [&](int64_t s) { return ((double)s * 0.0625) / (double)area <= thr; };
    if (!pred(0))
        return -1;
    int64_t lo = 0, hi = 1ll << 40;
    if (pred(hi))
        return hi;
    while (hi - lo > 1) {
        const int64_t mid = lo + (hi - lo) / 2;
        if (pred(mid))
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

} // namespace

struct frac_ctx {
    int device = 0;
    frac_params p{};
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::string err;

    HostPlane src, tgt;
    bool same_plane = true;
    bool planes_set = false;
    DBuf<uint8_t> d_src, d_tgt;
    // frac_set_frame_async (ABI 9): the frame after the current one is uploaded into d_src_next on copy_stream
    // while the context's stream still reads d_src; the two swap at the call (created on first use)
    DBuf<uint8_t> d_src_next;
    hipStream_t copy_stream = nullptr;
    hipEvent_t up_done = nullptr, next_free = nullptr;
    bool next_free_recorded = false;
    uint32_t d_sstride = 0, d_tstride = 0;

    std::vector<frac_grid_item> doms, ranges;
    bool doms_set = false, ranges_set = false;
    bool dirty = true;

    // prepared state
    int n = 0;               // range side (0: rectangular ranges or domains, the sampled form)
    uint32_t S = 0;          // domain side (width for rectangles)
    uint32_t nw = 0, nh = 0, Sw = 0, Sh = 0; // range and domain width / height
    bool virt = false;       // sampled form (fracenc_gen.hip): one pool row per (domain, transform)
    bool generic = false;    // sampled form with a range size no templated engine covers (gen_search)
    uint32_t Teff = 4;       // transforms the engines search per pool row (1 in the sampled form)
    uint32_t K2 = 0;         // dwords per pool row
    uint32_t G = 4, NG = 1;
    uint32_t npos = 0;                      // pool positions (= domains); d_porig maps them to domain indices
    std::vector<uint32_t> bucket_begin, bucket_end; // per bucket (category + 1): pool positions
    BucketLayout layout{};                  // per-bucket counts and offsets (fracenc_bucket.hip); VALU slots
    BucketLayout mlayout{};                 // the same with the MFMA engine's 32-slot blocks and tiles
    uint32_t nvslots = 0;                   // VALU engine: range slots (64 per wave)
    bool doms_uploaded = false;             // d_doms holds c->doms
    bool doms_trusted = false;              // c->doms built by this library (quadtree levels): not re-validated
    bool ranges_dev = false;                // d_ranges was filled on the device (quadtree level): nr_dev items of n_dev
    uint32_t nr_dev = 0, n_dev = 0;
    std::vector<uint32_t> h_rkey, h_porig;  // frac_fetch: per-range bucket, pool order (classifier stats)
    std::vector<uint4> work;
    int64_t hitH = -1;
    bool all_fallback = false;
    std::vector<uint32_t> fb_iota;

    DBuf<frac_grid_item> d_doms, d_ranges;
    DBuf<uint32_t> d_porig, d_pool, d_fb_list, d_fb_count;
    // fallback_grid's per-listed-range scratch: the least key so far and the jobs done; all-ones / zero between
    // runs (the last job of a range resets its pair), set so when (re)allocated
    DBuf<unsigned long long> d_fb_key;
    DBuf<uint32_t> d_fb_done;
    // a fused resolver's fp32-regime ranges are listed, not evaluated: fallback_grid settles them before the
    // run's records are read (settle_fallback; frac_fetch launches it only when a range was listed)
    bool fb_pending = false;
    int fb_n = 0;
    FallbackArgs fb_args{};
    DBuf<int32_t> d_negsd2, d_slot_range;
    DBuf<uint4> d_work;
    DBuf<uint2> d_rbucket;
    DBuf<uint32_t> d_rord, d_rkey;           // bucket-sorted range order; per range bucket
    DBuf<uint32_t> d_bk_keys, d_bk_keys2, d_bk_iota, d_bk_first, d_bk_err, d_bk_cnt;
    DBuf<uint16_t> d_bsum_s, d_bsum_t; // the source / target plane's block sums (frame_block_sums)
    DBuf<uint8_t> d_bk_tmp;
    size_t bk_tmp_bytes = 0;
    DBuf<unsigned long long> d_best_key;
    DBuf<frac_encode_item> d_out;
    DBuf<RangeAux> d_aux;

    // MFMA engine layout
    uint32_t engine = FRAC_ENGINE_VALU;    // engine chosen for the current geometry
    uint32_t nblocks = 0, ntiles = 0;
    std::vector<uint4> m_work;             // per WG (4 range blocks: search_mfma)
    std::vector<uint32_t> m_blk_ptr, m_blk_ent;
    std::vector<uint4> m8_work;            // per WG (8 range blocks: search_dft; m8_bpw for the 16-wave forms)
    uint32_t m8_bpw = 8;                   // range blocks per workgroup of m8_work
    // T = 8 on the Fourier path (n = 8, ratio 2): Flip_Rotate_k = Flip ∘ Rotate_k (image/transform.h:32-41),
    // so the flip half is the rotation search of each range read through Flip — a second copy of every
    // range block (blocks nblocks .. 2·nblocks − 1, same bucket), resolved together with the original
    // (resolve_dft: Rotate-group index t' of the flipped copy = transform 4 + (−t' mod 4))
    uint32_t dft_copies = 1;
    std::vector<uint32_t> m8_blk_ptr, m8_blk_ent;
    DBuf<uint4> d_m8_work;
    DBuf<uint32_t> d_m8_blk_ptr, d_m8_blk_ent;
    DBuf<int32_t> d_m_slot_range, d_m_tile_pos;
    DBuf<uint32_t> d_m_range_slot, d_m_blk_ptr, d_m_blk_ent, d_m_rconst, d_m_dconst;
    DBuf<uint4> d_m_work, d_m_dtiles, d_m_rfrags;
    DBuf<uint2> d_m_entries;

    // decoder state
    DBuf<uint8_t> d_dec_src, d_dec_tgt, d_color;
    DBuf<unsigned long long> d_dec_part;
    DBuf<DecodeState> d_dec_state;
    DecodeState* h_dec_state = nullptr;
    DBuf<uint2> d_dft_tguard;
    DBuf<int32_t> d_dft_trmax; // the six-MFMA fast path's per-tile R6 threshold (kDftFast6)
    DBuf<uint32_t> d_dft_tpool; // pool rows in tile order (resolve_dft)
    DBuf<uint32_t> d_dft_rorb;  // range pixel pairs in orbit order, per slot (resolve_dft)
    DBuf<frac_qt_leaf> d_qt_leaves32; // frac_encode_quadtree_leaves' device-side leaves (pageable caller buffer)
    DBuf<unsigned long long> d_dft_slotbest; // per slot the search's merged word (search_dft → resolve_dft,
                                             // search_mfma n ≤ 4 → resolve_small)
    DBuf<uint4> d_rstat;        // per range: the winner's sums (resolve_dft → fit_rstat)
    DBuf<frac_grid_item> d_cls_items;
    DBuf<uint32_t> d_cls_list;
    DBuf<int32_t> d_cls_out;
    DBuf<uint32_t> d_dft_rguard;
    // SEA engine: sort keys/values (double-buffered for the radix sort), sorted entries
    DBuf<uint32_t> d_sea_dkey, d_sea_dkey2, d_sea_dpos, d_sea_dpos2, d_sea_rkey, d_sea_rkey2, d_sea_rord,
        d_sea_rord2, d_sea_bend, d_sea_spool;
    DBuf<SeaEntry> d_sea_ent;
    DBuf<int32_t> d_sea_snegsd2;
    DBuf<frac_tuple> d_tuples; // frac_fetch_tuples staging
    frac_tuple* tuple_sink = nullptr; // frac_set_tuple_sink: every frac_run's tuples also go here
    // SEA engine, tiled form (fracenc_tp.hip)
    bool tp = false;
    TpBuckets tp_bk{};
    std::vector<uint4> tp_groups;
    uint32_t tp_key_bits = 16; // (bucket << 16 | Σ) sort keys: 16 + ⌈log2 nb⌉ bits
    std::vector<uint32_t> tp_iota;
    std::vector<uint2> tp_blk_group;
    DBuf<uint4> d_tp_groups;
    DBuf<uint2> d_tp_blk_group, d_tp_tile_sd, d_tp_blk_sr;
    DBuf<uint32_t> d_tp_blk_u, d_tp_nch, d_tp_choff, d_tp_blkcnt, d_tp_tot, d_tp_iota, d_tp_pairs, d_tp_row_of;
    DBuf<int32_t> d_tp_rbk;
    DBuf<uint8_t> d_tp_tmp;
    size_t tp_tmp_bytes = 0;
    DBuf<Frc1MinMax> d_frc_mm;             // frac_pack_frc1
    DBuf<unsigned long long> d_frc_rec;
    DBuf<uint32_t> d_frc_words;
    std::vector<frac_encode_item> qt_res; // quadtree: one level's results (kept: no page faults per call)
    // quadtree: the per-level domain grids (geometry only) of the last frame size, by log2(n)
    uint32_t qt_w = 0, qt_h = 0;
    std::vector<frac_grid_item> qt_doms[5];
    DBuf<frac_grid_item> qt_ddoms[5];     // their device copies
    DBuf<frac_grid_item> d_qt_next;       // the next level's ranges, built on the device
    DBuf<frac_encode_item> d_qt_leaves;   // the frame's leaves, in output order
    DBuf<uint32_t> d_qt_flags, d_qt_offs, d_qt_count;
    DBuf<unsigned long long> d_qt_stats; // quadtree: the levels' frac_stats counters (qt_level_stats)
    // device-planned quadtree levels (frac_encode_quadtree, MFMA engine): the levels' plans (+1 for
    // the count after the last), their bucket bounds, and the first level's range grid
    DBuf<DevPlan> d_qt_plan;
    QtFrameSum* h_qt_sum = nullptr; // pinned, mapped: qt_finish writes the frame's counts there
    DBuf<uint32_t> d_qt_first;
    DBuf<frac_grid_item> d_qt_r0;
    uint32_t qt_r0_key[3] = {0, 0, 0};
    const DevPlan* qplan = nullptr; // set while a device-planned level launches (launch_all in plan mode)
    uint32_t qp_nwork_cap = 0;      // its work-item bound: the search grid
    DBuf<uint8_t> d_qt_tmp;
    size_t qt_tmp_bytes = 0;
    bool qt_dvalid[5] = {false, false, false, false, false};
    DBuf<uint8_t> d_sea_tmp;
    DBuf<unsigned long long> d_sea_count; // candidates the SEA search evaluated
    uint64_t eligible_pairs = 0;          // Σ over ranges of its bucket's domain count
    uint64_t evaluated_ran = 0;           // frac_stats.evaluated_mappings of the last run
    size_t sea_tmp_bytes = 0;
    DBuf<frac_encode_item> d_dec_items;
    DBuf<unsigned long long> d_dec_sum;
    unsigned long long* h_dec_sum = nullptr; // pinned

    std::vector<RangeAux> h_aux;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    hipEvent_t handoff = nullptr; // frac_set_stream: the new stream waits for the old one's work (created on use)
    // FRAC_FLAG_TIMING: the same four boundaries (start | prep | search | finish) of every run
    // since the last frac_timing_history call, a ring of kHistRuns runs (created on first use)
    std::vector<hipEvent_t> hist;
    uint64_t hist_runs = 0, hist_read = 0;
    int prep_knobs = -1; // FRAC_MFMA_VARIANT / FRAC_MFMA_DFT as of the last prepare (frac_run)
    int mfma_var_ran = 0; // the schedule variant search_mfma last ran with (its entry layout)
    bool ran = false;
    uint32_t engine_ran = FRAC_ENGINE_VALU;
    uint32_t form_ran = FRAC_FORM_DOT2;
    bool fit_rstat = false; // resolve_dft recorded the winners' sums (fit_rstat instead of fit_winner)
    bool fit_fused = false; // resolve_dft wrote the records itself (no fit launch)
    uint64_t flops_ran = 0;

    int fail(int code, const std::string& msg)
    {
        err = msg;
        g_last_error = msg;
        return code;
    }
    int hip(hipError_t e, const char* what)
    {
        if (e == hipSuccess)
            return FRAC_OK;
        return fail(FRAC_E_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
    }
};

// ranges of the current search: the caller's list, or (quadtree levels) a list the device built
inline size_t nranges(const frac_ctx* c) { return c->ranges_dev ? c->nr_dev : c->ranges.size(); }

#define FRAC_TRY(expr)                                                                                                 \
    do {                                                                                                               \
        int _rc = (expr);                                                                                              \
        if (_rc != FRAC_OK)                                                                                            \
            return _rc;                                                                                                \
    } while (0)
#define FRAC_HIP(ctx, expr) FRAC_TRY((ctx)->hip((expr), #expr))

namespace {
constexpr uint32_t kHistRuns = 256;

// Boundary k of the current run (0 start, 1 search begins, 2 search ends, 3 finish ends), one
// event each: the run's slot in the timing history (frac_timing_history), which frac_stats reads
// for the last run (last_event).  Every record is a marker packet the GPU waits on, so a second
// record per boundary cost C2 (Lenna 512², T = 8) ≈ 17 µs per frame.
// Boundaries 0–2 only time the chain: their markers skip the system-scope fence (a cache write-back
// and invalidate per marker, and the next kernel starting on a cold L2).  Boundary 3 ends the run
// and keeps the default fence, so a host that synchronises on the stream still sees every write.
hipError_t create_timing_event(hipEvent_t* e, size_t k)
{
    return (k % 4) == 3 ? hipEventCreate(e) : hipEventCreateWithFlags(e, hipEventDisableSystemFence);
}

int mark_event(frac_ctx* c, int k)
{
    hipEvent_t e = c->hist.empty() ? c->ev[k] : c->hist[(size_t)(c->hist_runs % kHistRuns) * 4 + k];
    FRAC_HIP(c, hipEventRecord(e, c->stream));
    return FRAC_OK;
}

// boundary k of the last completed launch (after launch_all / launch_generic counted it)
hipEvent_t last_event(const frac_ctx* c, int k)
{
    if (c->hist.empty() || c->hist_runs == 0)
        return c->ev[k];
    return c->hist[(size_t)((c->hist_runs - 1) % kHistRuns) * 4 + k];
}
} // namespace

namespace {

int check_params(const frac_params* p, std::string& msg)
{
    if (!p) {
        msg = "params is NULL";
        return FRAC_E_INVALID;
    }
    if (p->transforms != 4 && p->transforms != 8) {
        msg = "transforms must be 4 or 8";
        return FRAC_E_INVALID;
    }
    if (p->engine > FRAC_ENGINE_SEA) {
        msg = "unknown engine";
        return FRAC_E_INVALID;
    }
    if (p->flags & ~(FRAC_FLAG_TIMING | FRAC_FLAG_DIRECT_FORM | FRAC_FLAG_SEA_PER_RANGE | FRAC_FLAG_DECODE_STEPWISE)) {
        msg = "unknown flag bits";
        return FRAC_E_INVALID;
    }
    return FRAC_OK;
}

// The A/B knobs of the tuning build.  A product build compiles only the shipped forms (the
// alternative exact forms are frac_params flags), so it refuses a run with any of these set rather
// than silently running the default: encode(), the C++ EncodingEngineCore and the reference-side
// binding cannot be steered into an A/B form by the environment.
constexpr const char* kAbKnobs[] = {"FRAC_MFMA_VARIANT", "FRAC_MFMA_DFT", "FRAC_DFT_WGS", "FRAC_XCD_ORDER",
                                    "FRAC_SEA_TILED", "FRAC_DECODE_UNFUSED"};

// the knob's value in a tuning build; nullptr in a product build (check_ab_knobs refused it)
inline const char* ab_knob(const char* name) { return kTuningBuild ? getenv(name) : nullptr; }

int check_ab_knobs(std::string& msg)
{
    if (kTuningBuild)
        return FRAC_OK;
    for (const char* k : kAbKnobs) {
        const char* v = getenv(k);
        if (v && *v) {
            msg = std::string(k) + "=" + v + ": A/B knobs exist only in a -DFRAC_TUNING build (tools/build_tuning.py); "
                                             "the alternative exact forms are frac_params flags";
            return FRAC_E_INVALID;
        }
    }
    return FRAC_OK;
}

// FRAC_TRACE=1: host wall-clock of the preparation and quadtree phases on stderr (tuning aid)
struct HostTrace {
    bool on;
    const char* what;
    std::chrono::steady_clock::time_point t0, t;
    explicit HostTrace(const char* w) : on(getenv("FRAC_TRACE") != nullptr), what(w)
    {
        t0 = t = std::chrono::steady_clock::now();
    }
    void mark(const char* phase)
    {
        if (!on)
            return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[frac %s] %-22s %8.3f ms (total %8.3f)\n", what, phase,
                std::chrono::duration<double, std::milli>(now - t).count(),
                std::chrono::duration<double, std::milli>(now - t0).count());
        t = now;
    }
};

// Categories of items[list[k]] on the device plane (classify_items); synchronous.
int classify_on_device(frac_ctx* c, const std::vector<frac_grid_item>& items, const std::vector<uint32_t>& list,
                       const uint8_t* dplane, uint32_t dstride, std::vector<int32_t>& out)
{
    out.assign(list.size(), -1);
    if (list.empty())
        return FRAC_OK;
    HostTrace tr("classify");
    FRAC_HIP(c, c->d_cls_items.ensure(items.size()));
    FRAC_HIP(c, c->d_cls_list.ensure(list.size()));
    FRAC_HIP(c, c->d_cls_out.ensure(list.size()));
    FRAC_HIP(c, hipMemcpyAsync(c->d_cls_items.ptr, items.data(), items.size() * sizeof(frac_grid_item),
                               hipMemcpyHostToDevice, c->stream));
    FRAC_HIP(c, hipMemcpyAsync(c->d_cls_list.ptr, list.data(), list.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                               c->stream));
    ClassifyArgs a;
    a.plane = dplane;
    a.stride = dstride;
    a.items = c->d_cls_items.ptr;
    a.list = c->d_cls_list.ptr;
    a.n = (uint32_t)list.size();
    a.out = c->d_cls_out.ptr;
    tr.mark("alloc + H2D");
    classify_items<<<(unsigned)((list.size() + 3) / 4), 256, 0, c->stream>>>(a);
    FRAC_HIP(c, hipGetLastError());
    tr.mark("launch");
    FRAC_HIP(c, hipMemcpyAsync(out.data(), c->d_cls_out.ptr, list.size() * sizeof(int32_t), hipMemcpyDeviceToHost,
                               c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    tr.mark("D2H + sync");
    return FRAC_OK;
}

// the caller's plane straight to the device (no host copy): pageable memory, so the copy is
// complete, and the caller's buffer free again, when the call returns
int upload_plane(frac_ctx* c, const uint8_t* p, uint32_t w, uint32_t h, uint32_t stride, DBuf<uint8_t>& d,
                 uint32_t& dstride)
{
    dstride = (w + 63u) & ~63u;
    // one extra row + column of slack: kernels never read it, but keeps every 2×2 read in-bounds
    FRAC_HIP(c, d.ensure((size_t)dstride * (h + 1)));
    if (h == 0 || w == 0)
        return FRAC_OK;
    if (stride == dstride) // rows already at the device pitch: one linear copy (a 2-D copy is a slower path)
        FRAC_HIP(c, hipMemcpyAsync(d.ptr, p, (size_t)stride * (h - 1) + w, hipMemcpyHostToDevice, c->stream));
    else
        FRAC_HIP(c, hipMemcpy2DAsync(d.ptr, dstride, p, stride, w, h, hipMemcpyHostToDevice, c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    return FRAC_OK;
}

// The classifier keys of a run or a quadtree level from the planes' block sums (bucket_keys_bs) when every
// item is at most 32 rows high (q ≤ 16): the source plane's pyramid, and the target's when it is another plane.
static int plane_block_sums(frac_ctx* c, BlockSums& bs, BlockSums& bt)
{
    FRAC_HIP(c, c->d_bsum_s.ensure(std::max<size_t>(bs_words(c->src.w, c->src.h), 1)));
    launch_block_sums(c->d_src.ptr, c->d_sstride, c->src.w, c->src.h, c->d_bsum_s.ptr, c->stream);
    bs = bs_layout(c->d_bsum_s.ptr, c->src.w, c->src.h);
    bt = bs;
    if (!c->same_plane) {
        FRAC_HIP(c, c->d_bsum_t.ensure(std::max<size_t>(bs_words(c->tgt.w, c->tgt.h), 1)));
        launch_block_sums(c->d_tgt.ptr, c->d_tstride, c->tgt.w, c->tgt.h, c->d_bsum_t.ptr, c->stream);
        bt = bs_layout(c->d_bsum_t.ptr, c->tgt.w, c->tgt.h);
    }
    return FRAC_OK;
}

// The classifier buckets on the device (fracenc_bucket.hip): d_porig (pool position → domain index),
// d_rord (ranges in bucket order), d_rkey (per range bucket); first[b] / rfirst[b] = the first pool
// position / bucket-sorted range of bucket b (b = 0..kMaxBuckets).  One small synchronous copy.
int device_buckets(frac_ctx* c, int nb, uint32_t* dfirst, uint32_t* rfirst)
{
    const uint32_t nd = (uint32_t)c->doms.size(), nr = (uint32_t)nranges(c);
    if (nb == 1) { // one bucket: the pool is the domain list, the ranges keep their order
        if (nd)
            fill_iota<<<(nd + 255) / 256, 256, 0, c->stream>>>(c->d_porig.ptr, nd);
        if (nr) {
            fill_iota<<<(nr + 255) / 256, 256, 0, c->stream>>>(c->d_rord.ptr, nr);
            FRAC_HIP(c, hipMemsetAsync(c->d_rkey.ptr, 0, nr * sizeof(uint32_t), c->stream));
        }
        for (int b = 0; b <= kMaxBuckets; ++b) {
            dfirst[b] = b == 0 ? 0u : nd;
            rfirst[b] = b == 0 ? 0u : nr;
        }
        return FRAC_OK;
    }
    HostTrace tr("buckets");
    const uint32_t m = std::max(std::max(nd, nr), 1u);
    FRAC_HIP(c, c->d_bk_keys.ensure(m));
    FRAC_HIP(c, c->d_bk_cnt.ensure((size_t)(2 * ((m + kBkTile - 1) / kBkTile) + 2) * kMaxBuckets));
    FRAC_HIP(c, c->d_bk_first.ensure(2 * (kMaxBuckets + 1) + 1));
    tr.mark("alloc");
    uint32_t* first = c->d_bk_first.ptr;
    uint32_t* err = first + 2 * (kMaxBuckets + 1);
    FRAC_HIP(c, hipMemsetAsync(err, 0, sizeof(uint32_t), c->stream));
    const uint8_t* tplane = c->same_plane ? c->d_src.ptr : c->d_tgt.ptr;
    const uint32_t tstride = c->same_plane ? c->d_sstride : c->d_tstride;
    // a stored −1 is classified on the item's own plane (Classifier2::compare, Classifier2.cpp:70-81);
    // the pool order porig and the bucket-sorted ranges rord by the stable bucket sort
    // both grids' keys, in one launch for the usual 2n → n geometry
    const KeySeg kd{c->d_doms.ptr, nd, c->d_src.ptr, c->d_sstride, c->d_bk_keys.ptr, nullptr, err, nullptr};
    const KeySeg kr{c->d_ranges.ptr, nr, tplane, tstride, c->d_rkey.ptr, nullptr, err, nullptr};
    if (c->Sh <= 32 && c->Sw <= 32 && c->nh <= 32 && c->nw <= 32) { // from the planes' block sums
        BlockSums bs, bt;
        FRAC_TRY(plane_block_sums(c, bs, bt));
        launch_bucket_keys_bs(kd, bs, c->Sw, c->Sh, kr, bt, c->nw, c->nh, c->stream);
    } else {
        launch_bucket_keys_pair(kd, c->Sh, kr, c->nh, c->stream);
    }
    const BkSeg sd = bk_seg_of(c->d_bk_keys.ptr, nd, nullptr, c->d_bk_cnt.ptr, first, c->d_porig.ptr);
    const BkSeg sr = bk_seg_of(c->d_rkey.ptr, nr, nullptr, c->d_bk_cnt.ptr + (size_t)sd.tiles * kMaxBuckets,
                               first + kMaxBuckets + 1, c->d_rord.ptr);
    launch_bucket_sorts(sd, sr, c->stream);
    uint32_t h[2 * (kMaxBuckets + 1) + 1];
    tr.mark("enqueue");
    FRAC_HIP(c, hipMemcpyAsync(h, first, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    tr.mark("D2H + sync");
    if (h[2 * (kMaxBuckets + 1)])
        return c->fail(FRAC_E_INVALID, "item category outside -1..5");
    for (int b = 0; b <= kMaxBuckets; ++b) {
        dfirst[b] = h[b];
        rfirst[b] = h[kMaxBuckets + 1 + b];
    }
    return FRAC_OK;
}

inline int mfma_variant(frac_ctx* c, int& var);
inline bool mfma_dft_enabled(const frac_ctx* c);
// the Fourier search variants that run 4-wave workgroups (and read m_work): 1, 3 and the odd
// ablations below 200; every other variant runs 8-wave workgroups on m8_work
// the variants that run search_dft in 4-wave workgroups over the 4-block work lists: 1, 3 and the
// tuning ablations of 1 (the other odd A/B values, e.g. 21, are 8-block forms)
inline bool dft_four_wave(int var)
{
    return var == 1 || var == 3 || var == 9 || var == 17 || var == 41 || var == 65 || var == 73 || var == 105;
}
// the Fourier form's domain/range fragment layout: 4 (8 MFMA per tile pair), 5 (kDft5, variants 20, 22),
// 6 (kDft6, variants 21, 23)
constexpr int kTpVar = 1 | kDftChain | (kDftTpForm == 6 ? kDft6 : 0); // the SEA tiled form's search_dft
constexpr uint32_t kTpKS = kDftTpForm == 4 ? 4u : 5u;                    // its domain fragments per tile
inline int dft_form(int var)
{
    if (var == 20 || var == 22)
        return 5;
    const bool six = var == 21 || var == 23 || (var >= 26 && var <= 28) || (var >= 33 && var <= 37) ||
                     var == 226 || var == 227 || (var >= 240 && var <= 243);
    return six ? 6 : 4;
}
// range blocks (waves) per workgroup of the Fourier search: 16 for variants 27 / 28 (1024-thread
// workgroups: each LDS stage serves twice the blocks, half the LDS-DMA per tile pair), else 8
inline uint32_t dft_bpw(int var) { return var == 27 || var == 28 ? 16u : kDftBlocksPerWG; }
// The Fourier path's own variants: 1, 3 (4-wave exact / guarded), 5 (8-tile stages), 6 (pairwise-tree
// row maximum), 12 (two range blocks per wave), 20 / 22 (five-MFMA form, packed / plain epilogue),
// 21 / 23 (six-MFMA form, one / two range blocks per wave), 24 (the 8-MFMA exact form in 8-wave
// workgroups), 26 (the six-MFMA form with the guarded constant-folded epilogue, kDftFast6) and the
// tuning ablations.  Every other value (the default, and the direct form's
// schedule knobs) runs kDftDefaultVariant.
// the six-MFMA form with the guarded constant-folded epilogue, the chunk unrolled and wave-uniform
// buffer_load … lds stages (variant 35): 12.09 / 12.02 vs 13.85 / 13.65 ms for the exact six-MFMA
// form (21) at C3 in two 8-round interleaved A/Bs on two boxes (profiles/r03/session3/r03_ab5.log,
// r03_ab6.log); 21 was 13.71 vs 15.23 ms for the 8-MFMA form (24) in round 2
constexpr int kDftDefaultVariant = 35;
// up to this many domain tiles the product build's search also carries the winning chunk's tile mask
// (search_dft TMASK; the tuning build's variant 37 always does)
constexpr uint32_t kDftTmaskTiles = 1024;
inline int dft_variant(int var)
{
    static const int own[] = {1, 3, 5, 6, 12, 20, 21, 22, 23, 24, 26, 27, 28, 33, 34, 35, 36, 37, 9, 17, 41, 65, 73, 105};
    for (int v : own)
        if (var == v)
            return var;
    return var >= 200 ? var : kDftDefaultVariant;
}

// Domain items as the search needs them: one size (Size32u, rectangles allowed), at least 2×2 (the
// sampler reads 2×2 blocks, image/sampler.h:21-38), inside the source plane once one is set.
// frac_set_domains runs it, so a reference-side engine rejects a bad grid in its constructor
// (EncodingEngine2.cpp:22-29 catches there), and prepare() again against the current plane.
int check_domains(frac_ctx* c, const frac_grid_item* d, size_t nd)
{
    if (!nd)
        return FRAC_OK;
    const uint32_t Sw = d[0].w, Sh = d[0].h;
    if (Sw < 2 || Sh < 2)
        return c->fail(FRAC_E_INVALID, "domain sides must be at least 2");
    if ((uint64_t)nd >= (1u << 24))
        return c->fail(FRAC_E_INVALID, "at most 2^24 - 1 domains");
    for (size_t i = 0; i < nd; ++i) {
        if (d[i].w != Sw || d[i].h != Sh)
            return c->fail(FRAC_E_INVALID, "all domains must be of one size");
        if (c->planes_set && ((uint64_t)d[i].x + d[i].w > c->src.w || (uint64_t)d[i].y + d[i].h > c->src.h))
            return c->fail(FRAC_E_INVALID, "domain outside the source plane");
        if (d[i].category < -1 || d[i].category > 5)
            return c->fail(FRAC_E_INVALID, "domain category must be -1..5");
    }
    return FRAC_OK;
}

// Rectangular items: under a rotation a rectangle's samples leave its own patch
// (image/transform.h:96-109 maps x' = y for Rotate_90 with the patch's own sizes), reading the plane
// around it.  The reference reads whatever is there, inside the image; beyond the image it reads out
// of bounds.  Every 2×2 block any transform samples — at the metric points (x·⌊Sw/nw⌋, y·⌊Sh/nh⌋) and
// the fit points ((x·Sw)/nw, (y·Sh)/nh), after the sampler's edge clamp — must lie inside the source
// plane for every domain; else the search is refused.
struct SampleBox {
    int x0 = INT32_MAX, x1 = INT32_MIN, y0 = INT32_MAX, y1 = INT32_MIN;
};
// the pixels (relative to the domain origin) that transform t's 2×2 samples of an Sw×Sh domain read
// for an nw×nh range: the metric points and/or the fit points, after the sampler's edge clamp
SampleBox sample_box(int t, int Sw, int Sh, int nw, int nh, bool metric, bool fit)
{
    // the sampler's own table (fracenc_common.h lut(), which gen_sample reads), so the refusal and
    // the decode check cannot drift from the samples the kernels take
    const Aff L = lut(t);
    const int a[8] = {L.a0, L.a1, L.a2, L.a3, L.a4, L.a5, L.a6, L.a7};
    SampleBox b;
    auto add = [&](int lx, int ly) {
        if (lx == Sw - 1)
            --lx;
        if (ly == Sh - 1)
            --ly;
        const int px = a[0] * lx + a[1] * ly + a[2] * (Sw - 1) + a[3] * (Sh - 1);
        const int py = a[4] * lx + a[5] * ly + a[6] * (Sw - 1) + a[7] * (Sh - 1);
        for (int k = 0; k < 4; ++k) {
            const int qx = px + (k & 1 ? a[0] : 0) + (k & 2 ? a[1] : 0);
            const int qy = py + (k & 1 ? a[4] : 0) + (k & 2 ? a[5] : 0);
            b.x0 = std::min(b.x0, qx);
            b.x1 = std::max(b.x1, qx);
            b.y0 = std::min(b.y0, qy);
            b.y1 = std::max(b.y1, qy);
        }
    };
    for (int y = 0; y < nh; ++y)
        for (int x = 0; x < nw; ++x) {
            if (metric)
                add(x * (Sw / nw), y * (Sh / nh));
            if (fit)
                add((x * Sw) / nw, (y * Sh) / nh);
        }
    return b;
}

bool box_inside(const SampleBox& b, uint32_t x, uint32_t y, uint32_t w, uint32_t h)
{
    return (int64_t)x + b.x0 >= 0 && (int64_t)x + b.x1 < (int64_t)w && (int64_t)y + b.y0 >= 0 &&
           (int64_t)y + b.y1 < (int64_t)h;
}

int check_rect_samples(frac_ctx* c)
{
    SampleBox u;
    for (uint32_t t = 0; t < c->p.transforms; ++t) {
        const SampleBox b = sample_box((int)t, (int)c->Sw, (int)c->Sh, (int)c->nw, (int)c->nh, true, true);
        u.x0 = std::min(u.x0, b.x0);
        u.x1 = std::max(u.x1, b.x1);
        u.y0 = std::min(u.y0, b.y0);
        u.y1 = std::max(u.y1, b.y1);
    }
    for (const auto& d : c->doms)
        if (!box_inside(u, d.x, d.y, c->src.w, c->src.h))
            return c->fail(FRAC_E_INVALID, "a transform of a rectangular domain samples outside the source plane "
                                           "(the reference reads out of bounds there)");
    return FRAC_OK;
}

int prepare(frac_ctx* c)
{
    HostTrace tr("prepare");
    if (!c->planes_set || !c->doms_set || !c->ranges_set)
        return c->fail(FRAC_E_STATE, "planes, domains and ranges must be set before frac_run");
    const uint32_t T = c->p.transforms;
    // geometry (TransformMatcher::matchTransformType, encode/transformmatcher.h:70-78): n×n ranges
    // and S×S domains, S > n (main.cpp:99 rejects target >= source).  S = 2n with n ∈ {2, 4, 8, 16}
    // is every engine's decimate-then-permute path; any other pair — the CLI default 16→4 among
    // them — runs the sampled form (fracenc_gen.hip): one pool row per (domain, transform).
    // ranges: one size nw × nh (Size32u items, image/partition2.hpp:13-31: rectangles allowed)
    const uint32_t nw = c->ranges_dev ? c->n_dev : c->ranges.empty() ? 8u : c->ranges[0].w;
    const uint32_t nh = c->ranges_dev ? c->n_dev : c->ranges.empty() ? 8u : c->ranges[0].h;
    for (const auto& r : c->ranges) {
        if (c->ranges_dev)
            break; // built on the device from validated parents (frac_encode_quadtree)
        if (r.w != nw || r.h != nh)
            return c->fail(FRAC_E_INVALID, "all ranges must be of one size");
        if ((uint64_t)r.x + r.w > c->tgt.w || (uint64_t)r.y + r.h > c->tgt.h)
            return c->fail(FRAC_E_INVALID, "range outside the target plane");
    }
    if (nw < 2 || nh < 2)
        return c->fail(FRAC_E_INVALID, "range sides must be at least 2");
    if ((uint64_t)nw * nh > (1ull << 26))
        return c->fail(FRAC_E_INVALID, "ranges of more than 2^26 pixels");
    // domains: validated by frac_set_domains (one size, inside the plane); re-checked against the
    // current plane, which may have changed since
    const uint32_t Sw = c->doms.empty() ? 2u * nw : c->doms[0].w;
    const uint32_t Sh = c->doms.empty() ? 2u * nh : c->doms[0].h;
    if (!c->doms_trusted)
        FRAC_TRY(check_domains(c, c->doms.data(), c->doms.size()));
    // RootMeanSquare's different-size branch (image/metrics.h:37-50) needs a domain wider than the
    // range (its FRAC_ASSERT, :39; main.cpp:99 for the CLI's square items)
    if (Sw <= nw)
        return c->fail(FRAC_E_INVALID, "domains must be wider than the ranges (metrics.h:39, main.cpp:99)");
    const bool square = nw == nh && Sw == Sh;
    const int n = square ? (int)nw : 0;
    const bool pow2 = n == 2 || n == 4 || n == 8 || n == 16;
    c->virt = !(pow2 && Sw == 2u * nw);
    c->generic = !pow2;
    c->S = Sw;
    c->nw = nw;
    c->nh = nh;
    c->Sw = Sw;
    c->Sh = Sh;
    if (!square)
        FRAC_TRY(check_rect_samples(c));
    c->Teff = c->virt ? 1u : T;
    c->K2 = (nw * nh + 1) / 2;
    if ((uint64_t)c->doms.size() * (c->virt ? T : 1u) >= (1u << 24))
        return c->fail(FRAC_E_INVALID, "at most 2^24 - 1 domains (domains x transforms in the sampled form)");
    c->n = n;
    c->G = c->virt ? 1u : (n == 16 ? 1u : (n <= 4 ? T : 4u));
    c->NG = c->virt ? 1u : T / c->G;

    tr.mark("validate");
    // buckets: category + 1 (0 = category −1) with the classifier, a single bucket without.  Every
    // per-item step runs on the device (device_buckets); the host works from the bucket counts.
    const int nb = c->p.use_classifier ? 7 : 1;
    const size_t nd = c->doms.size(), nr = nranges(c);
    auto up = [&](void* dst, const void* srcp, size_t bytes) {
        return bytes ? c->hip(hipMemcpyAsync(dst, srcp, bytes, hipMemcpyHostToDevice, c->stream), "upload") : 0;
    };
    FRAC_HIP(c, c->d_doms.ensure(nd));
    FRAC_HIP(c, c->d_ranges.ensure(nr));
    FRAC_HIP(c, c->d_porig.ensure(nd));
    FRAC_HIP(c, c->d_rord.ensure(nr));
    FRAC_HIP(c, c->d_rkey.ensure(nr));
    if (!c->doms_uploaded) {
        FRAC_TRY(up(c->d_doms.ptr, c->doms.data(), nd * sizeof(frac_grid_item)));
        c->doms_uploaded = true;
    }
    if (!c->ranges_dev)
        FRAC_TRY(up(c->d_ranges.ptr, c->ranges.data(), nr * sizeof(frac_grid_item)));
    uint32_t dfirst[kMaxBuckets + 1], rfirst[kMaxBuckets + 1];
    FRAC_TRY(device_buckets(c, nb, dfirst, rfirst));
    tr.mark("buckets (device)");
    c->npos = (uint32_t)nd;
    c->bucket_begin.assign(dfirst, dfirst + nb);
    c->bucket_end.assign(dfirst + 1, dfirst + nb + 1);
    std::vector<uint32_t> rbeg(rfirst, rfirst + nb + 1);
    // the engines' pool rows per bucket: pool positions, or T rows per position in the sampled form
    const uint32_t VT = c->virt ? T : 1u;
    std::vector<uint32_t> eb(nb), ee(nb);
    BucketLayout L{};
    L.nb = (uint32_t)nb;
    L.VT = VT;
    for (int b = 0; b < nb; ++b) {
        eb[b] = c->bucket_begin[b] * VT;
        ee[b] = c->bucket_end[b] * VT;
        L.dbeg[b] = c->bucket_begin[b];
        L.dcnt[b] = c->bucket_end[b] - c->bucket_begin[b];
        L.rbeg[b] = rbeg[b];
        L.rcnt[b] = rbeg[b + 1] - rbeg[b];
    }
    c->layout = L;
    // range slots: per bucket, padded to whole waves of 64 (the VALU engine's work lists only)
    c->work.clear();
    c->nvslots = 0;
    const bool valu_lists = c->p.engine == FRAC_ENGINE_VALU && !c->generic;
    std::vector<std::pair<uint32_t, int>> blocks; // (slot base, bucket)
    for (int b = 0; valu_lists && b < nb; ++b) {
        c->layout.slot_first[b] = c->nvslots; // used by the VALU slot fill below
        const uint32_t cnt = L.rcnt[b];
        for (uint32_t s0 = 0; s0 < cnt; s0 += 64)
            blocks.emplace_back(c->nvslots + s0, b);
        c->nvslots += (cnt + 63) / 64 * 64;
    }
    size_t total_blocks = 0;
    for (auto& bl : blocks)
        if (ee[bl.second] > eb[bl.second])
            total_blocks += c->NG;
    // domain splits: enough waves to fill 256 CUs several times over, ≥ 32 domains per wave
    const size_t target_waves = 8192;
    for (auto& bl : blocks) {
        const uint32_t b0 = eb[bl.second], b1 = ee[bl.second];
        const uint32_t D = b1 - b0;
        if (D == 0)
            continue;
        size_t splits = total_blocks ? (target_waves + total_blocks - 1) / total_blocks : 1;
        splits = std::min<size_t>(splits, std::max<uint32_t>(1u, D / 32u));
        splits = std::max<size_t>(splits, 1);
        for (uint32_t g = 0; g < c->NG; ++g)
            for (size_t s = 0; s < splits; ++s) {
                const uint32_t pb = b0 + (uint32_t)((uint64_t)D * s / splits);
                const uint32_t pe = b0 + (uint32_t)((uint64_t)D * (s + 1) / splits);
                if (pe > pb)
                    c->work.push_back(make_uint4(bl.first, pb, pe, g));
            }
    }
    tr.mark("buckets + valu work");
    c->eligible_pairs = 0;
    for (int b = 0; b < nb; ++b)
        c->eligible_pairs += (uint64_t)L.rcnt[b] * L.dcnt[b];
    c->hitH = compute_hit_limit(c->p.rms_threshold, Sw * Sh); // the domain's area (image/metrics.h:49)
    // every candidate in the reference's fp32 arithmetic (gen_fallback): with a threshold no exact error can
    // meet, and for range sides above kGenMaxN, whose S16 outgrows the search keys' error field — there the
    // exact search could not order the candidates, and S16 ≥ 2^24 is the fp32 regime anyway for almost all
    c->all_fallback = c->hitH >= kExactLimit || nw > kGenMaxN || nh > kGenMaxN;

    // engine.  MFMA: exact for every templated n (n = 16 through search_mfma16's integer epilogue).
    // SEA covers n ≤ 8 (its exact evaluation holds a candidate in one wave's VGPRs): larger ranges run
    // the exhaustive MFMA search, which gives the same records.  Range sizes without a templated
    // engine run gen_search (VALU) whatever the request.
    c->engine = c->generic                                ? FRAC_ENGINE_VALU
                : c->p.engine == FRAC_ENGINE_VALU          ? FRAC_ENGINE_VALU
                : c->p.engine == FRAC_ENGINE_SEA && n <= 8 ? FRAC_ENGINE_SEA
                                                           : FRAC_ENGINE_MFMA;
    // SEA, n = 8, T = 4: the tiled form (FRAC_FLAG_SEA_PER_RANGE keeps the per-range form; in a
    // tuning build also FRAC_SEA_TILED=0)
    {
        const char* st = ab_knob("FRAC_SEA_TILED");
        c->tp = c->engine == FRAC_ENGINE_SEA && !c->virt && n == 8 && T == 4 &&
                !(c->p.flags & FRAC_FLAG_SEA_PER_RANGE) && (st ? atoi(st) != 0 : true);
    }
    if (c->tp) {
        if (nb > kTpMaxBuckets)
            return c->fail(FRAC_E_INVALID, "SEA: too many classifier buckets");
        TpBuckets& bk = c->tp_bk;
        bk = TpBuckets{};
        bk.nb = (uint32_t)nb;
        uint32_t nt = 0, nbk = 0;
        for (int b = 0; b < nb; ++b) {
            bk.dom_begin[b] = c->bucket_begin[b];
            bk.dom_count[b] = c->bucket_end[b] - c->bucket_begin[b];
            bk.tile_first[b] = nt;
            bk.tile_count[b] = (bk.dom_count[b] + 31) / 32;
            nt += bk.tile_count[b];
            bk.rng_begin[b] = rbeg[b];
            bk.rng_count[b] = rbeg[b + 1] - rbeg[b];
            bk.blk_first[b] = nbk;
            bk.blk_count[b] = (bk.rng_count[b] + 31) / 32;
            nbk += bk.blk_count[b];
        }
        if (nt >= (1u << 28)) // chunk entries hold the tile in 28 bits (search_dft CHUNKED)
            return c->fail(FRAC_E_INVALID, "SEA: too many domain tiles");
        c->ntiles = nt;
        c->nblocks = nbk;
        c->tp_key_bits = 16;
        while ((1u << (c->tp_key_bits - 16)) < (uint32_t)nb)
            ++c->tp_key_bits;
        c->tp_groups.clear();
        c->tp_blk_group.assign(nbk, make_uint2(0xffffffffu, 0u));
        for (int b = 0; b < nb; ++b) {
            if (!bk.tile_count[b])
                continue; // no domain: the bucket's ranges keep the default record
            for (uint32_t g0 = 0; g0 < bk.blk_count[b]; g0 += kDftBlocksPerWG) {
                const uint32_t gi = (uint32_t)c->tp_groups.size();
                const uint32_t nbl = std::min(kDftBlocksPerWG, bk.blk_count[b] - g0);
                c->tp_groups.push_back(make_uint4(bk.blk_first[b] + g0, nbl, bk.tile_first[b], bk.tile_count[b]));
                for (uint32_t k = 0; k < nbl; ++k)
                    c->tp_blk_group[bk.blk_first[b] + g0 + k] = make_uint2(gi, k);
            }
        }
    }
    c->dft_copies = 1;
    if (c->engine == FRAC_ENGINE_MFMA) {
        // range blocks of 32 slots per bucket; domain tiles of 32 engine pool rows per bucket (the
        // maps themselves are filled on the device below)
        std::vector<uint32_t> blk_first(nb, 0), blk_count(nb, 0), tile_first(nb, 0), tile_count(nb, 0);
        uint32_t nbk = 0, nt = 0;
        for (int b = 0; b < nb; ++b) {
            blk_first[b] = nbk;
            blk_count[b] = (L.rcnt[b] + 31) / 32;
            nbk += blk_count[b];
            tile_first[b] = nt;
            tile_count[b] = (ee[b] - eb[b] + 31) / 32;
            nt += tile_count[b];
        }
        c->nblocks = nbk;
        c->ntiles = nt;
        c->mlayout = L;
        for (int b = 0; b < nb; ++b) {
            c->mlayout.slot_first[b] = 32 * blk_first[b];
            c->mlayout.tile_first[b] = tile_first[b];
        }
        // work items: groups of up to BPW blocks of one bucket × splits of its tiles, plus the
        // CSR map block → entry bases (work·BPW + wave) the resolve kernels read
        auto build_work = [&](uint32_t bpw, size_t target_wgs, std::vector<uint4>& work,
                              std::vector<uint32_t>& blk_ptr, std::vector<uint32_t>& blk_ent, bool xcd_order) {
            std::vector<uint32_t> split_of; // domain split of each work item
            // splits per bucket in proportion to its tiles, so every work item covers about
            // (groups × tiles) / target_wgs group-tiles — an equal count per bucket gave the small
            // buckets' items a few tiles each (their fixed cost of loading B fragments dominating) and
            // the large buckets' long ones the tail; Σ groups_b·splits_b ≤ target_wgs + groups
            uint64_t gtiles = 0;
            for (int b = 0; b < nb; ++b)
                if (tile_count[b])
                    gtiles += (uint64_t)((blk_count[b] + bpw - 1) / bpw * c->dft_copies) * tile_count[b];
            // every block of bucket b gets one entry per domain split of b: the CSR map is
            // sized by a count pass, then filled in work order (no per-block lists)
            const uint32_t ncp = c->dft_copies, nbt = c->nblocks * ncp; // T = 8 Fourier: flipped copies
            std::vector<uint32_t> nsplit(nb, 0);
            blk_ptr.assign(nbt + 1, 0);
            for (int b = 0; b < nb; ++b) {
                if (!tile_count[b] || !blk_count[b])
                    continue;
                const uint64_t tw = work_target(target_wgs, gtiles);
                size_t splits = gtiles ? (size_t)((tw * tile_count[b] + gtiles - 1) / gtiles) : 1;
                splits = std::max<size_t>(1, std::min<size_t>(splits, std::max<uint32_t>(1u, tile_count[b] / 4u)));
                uint32_t ns = 0;
                for (size_t sp = 0; sp < splits; ++sp)
                    ns += (uint64_t)tile_count[b] * (sp + 1) / splits > (uint64_t)tile_count[b] * sp / splits;
                nsplit[b] = (uint32_t)splits;
                for (uint32_t cp = 0; cp < ncp; ++cp)
                    for (uint32_t k = 0; k < blk_count[b]; ++k)
                        blk_ptr[cp * c->nblocks + blk_first[b] + k + 1] = ns;
            }
            for (uint32_t b = 0; b < nbt; ++b)
                blk_ptr[b + 1] += blk_ptr[b];
            blk_ent.assign(blk_ptr[nbt], 0);
            std::vector<uint32_t> cur(blk_ptr.begin(), blk_ptr.end() - 1);
            work.clear();
            for (uint32_t cp = 0; cp < ncp; ++cp)
                for (int b = 0; b < nb; ++b) {
                    if (!nsplit[b])
                        continue;
                    const size_t splits = nsplit[b];
                    const uint32_t bf = cp * c->nblocks + blk_first[b];
                    for (uint32_t g = 0; g < blk_count[b]; g += bpw) {
                        const uint32_t nbk = std::min(bpw, blk_count[b] - g);
                        for (size_t sp = 0; sp < splits; ++sp) {
                            const uint32_t t0 = tile_first[b] + (uint32_t)((uint64_t)tile_count[b] * sp / splits);
                            const uint32_t t1 = tile_first[b] + (uint32_t)((uint64_t)tile_count[b] * (sp + 1) / splits);
                            if (t1 <= t0)
                                continue;
                            const uint32_t w = (uint32_t)work.size();
                            work.push_back(make_uint4(bf + g, nbk, t0, t1));
                            split_of.push_back((uint32_t)sp);
                            for (uint32_t k = 0; k < nbk; ++k)
                                blk_ent[cur[bf + g + k]++] = w * bpw + k;
                        }
                    }
                }
            if (xcd_order && !work.empty()) {
                // XCD-aware order: workgroup n runs on XCD n % 8 (dispatch round-robin), so the
                // items of one domain split go to the same XCDs and their in-flight workgroups
                // stream the same tiles through that XCD's L2 together
                constexpr uint32_t kXcd = 8;
                std::vector<std::vector<uint32_t>> q(kXcd);
                uint32_t S = 0;
                for (uint32_t sp : split_of)
                    S = std::max(S, sp + 1);
                // split s → XCDs x ≡ s (mod S) when S ≤ 8 (round-robin over them), else XCD s mod 8
                std::vector<uint32_t> rr(S, 0);
                for (uint32_t w = 0; w < (uint32_t)work.size(); ++w) {
                    const uint32_t sp = split_of[w];
                    uint32_t x = sp % kXcd;
                    if (S <= kXcd) {
                        const uint32_t nx = (kXcd - 1 - sp) / S + 1; // XCDs sp, sp + S, ... below 8
                        x = sp + S * (rr[sp]++ % nx);
                    }
                    q[x].push_back(w);
                }
                std::vector<uint32_t> order;
                order.reserve(work.size());
                std::vector<size_t> head(kXcd, 0);
                while (order.size() < work.size()) {
                    bool any = false;
                    for (uint32_t x = 0; x < kXcd; ++x)
                        if (head[x] < q[x].size()) {
                            order.push_back(q[x][head[x]++]);
                            any = true;
                        } else { // an empty queue: keep the slot's XCD busy with another split
                            for (uint32_t y = 0; y < kXcd; ++y)
                                if (head[y] < q[y].size()) {
                                    order.push_back(q[y][head[y]++]);
                                    any = true;
                                    break;
                                }
                        }
                    if (!any)
                        break;
                }
                std::vector<uint32_t> inv(work.size());
                std::vector<uint4> nw(work.size());
                for (uint32_t n = 0; n < (uint32_t)order.size(); ++n) {
                    nw[n] = work[order[n]];
                    inv[order[n]] = n;
                }
                work.swap(nw);
                for (uint32_t& e : blk_ent)
                    e = inv[e / bpw] * bpw + e % bpw;
            }
        };
        const bool fourier = n == 8 && (T == 4 || T == 8) && !c->virt && mfma_dft_enabled(c);
        c->dft_copies = fourier && T == 8 ? 2u : 1u;
        int var = 0;
        FRAC_TRY(mfma_variant(c, var));
        const bool four_wave = dft_four_wave(var);
        if (n == 16) // search_mfma16: mfma16_bpw(T) range blocks per 4-wave workgroup
            build_work(mfma16_bpw(c->Teff), kMfma16TargetWgs, c->m_work, c->m_blk_ptr, c->m_blk_ent, false); // Teff: 1 when sampled
        else if (!fourier || four_wave) // the 8-wave Fourier search reads only its own list
            build_work(4, 8192, c->m_work, c->m_blk_ptr, c->m_blk_ent, false);
        else {
            c->m_work.clear();
            c->m_blk_ptr.assign(c->nblocks + 1, 0);
            c->m_blk_ent.clear();
        }
        if (n == 8 && !c->virt && (T == 4 || c->dft_copies == 2)) {
            // FRAC_DFT_WGS (tuning knob): target workgroup count of the Fourier search
            const char* tw = ab_knob("FRAC_DFT_WGS");
            c->m8_bpw = dft_bpw(dft_variant(var));
            const size_t wgs = tw ? (size_t)std::max(1, atoi(tw)) : 8192 / c->m8_bpw * 4;
            // FRAC_XCD_ORDER (tuning knob): 0 = work items in (block group, split) order
            const char* xo = ab_knob("FRAC_XCD_ORDER");
            build_work(c->m8_bpw, wgs, c->m8_work, c->m8_blk_ptr, c->m8_blk_ent, xo ? atoi(xo) != 0 : true);
        }
        else {
            c->m8_work.clear();
            c->m8_blk_ptr.clear();
            c->m8_blk_ent.clear();
        }
    }

    tr.mark("engine work");
    const size_t P = (size_t)c->npos * VT; // engine pool rows
    FRAC_HIP(c, c->d_pool.ensure(P * (size_t)c->K2));
    FRAC_HIP(c, c->d_negsd2.ensure(P));
    FRAC_HIP(c, c->d_slot_range.ensure(c->nvslots));
    FRAC_HIP(c, c->d_work.ensure(c->work.size()));
    FRAC_HIP(c, c->d_rbucket.ensure(nr));
    FRAC_HIP(c, c->d_best_key.ensure(nr));
    FRAC_HIP(c, c->d_out.ensure(nr));
    FRAC_HIP(c, c->d_aux.ensure(nr));
    FRAC_HIP(c, c->d_fb_list.ensure(nr));
    FRAC_HIP(c, c->d_fb_count.ensure(1));
    FRAC_TRY(up(c->d_work.ptr, c->work.data(), c->work.size() * sizeof(uint4)));
    if (nr)
        fill_rbucket<<<(unsigned)((nr + 255) / 256), 256, 0, c->stream>>>(L, c->d_rkey.ptr, (uint32_t)nr,
                                                                         c->d_rbucket.ptr);
    if (c->nvslots)
        fill_range_slots<<<(c->nvslots + 255) / 256, 256, 0, c->stream>>>(c->layout, c->d_rord.ptr, c->nvslots,
                                                                          c->d_slot_range.ptr, nullptr);
    if (c->all_fallback && nr)
        fill_iota<<<(unsigned)((nr + 255) / 256), 256, 0, c->stream>>>(c->d_fb_list.ptr, (uint32_t)nr);
    if (c->engine == FRAC_ENGINE_SEA) {
        if (c->bucket_end.size() > (size_t)kSeaMaxBuckets)
            return c->fail(FRAC_E_INVALID, "SEA: too many classifier buckets");
        FRAC_HIP(c, c->d_sea_dkey.ensure(std::max<size_t>(P, 1)));
        FRAC_HIP(c, c->d_sea_dkey2.ensure(std::max<size_t>(P, 1)));
        FRAC_HIP(c, c->d_sea_dpos.ensure(std::max<size_t>(P, 1)));
        FRAC_HIP(c, c->d_sea_dpos2.ensure(std::max<size_t>(P, 1)));
        FRAC_HIP(c, c->d_sea_ent.ensure(std::max<size_t>(P, 1)));
        FRAC_HIP(c, c->d_sea_snegsd2.ensure(std::max<size_t>(P, 1)));
        FRAC_HIP(c, c->d_sea_spool.ensure(std::max<size_t>(P * (size_t)(n * n / 2), 1)));
        FRAC_HIP(c, c->d_sea_rkey.ensure(std::max<size_t>(nr, 1)));
        FRAC_HIP(c, c->d_sea_rkey2.ensure(std::max<size_t>(nr, 1)));
        FRAC_HIP(c, c->d_sea_rord.ensure(std::max<size_t>(nr, 1)));
        FRAC_HIP(c, c->d_sea_rord2.ensure(std::max<size_t>(nr, 1)));
        FRAC_HIP(c, c->d_sea_bend.ensure(kSeaMaxBuckets));
        FRAC_HIP(c, c->d_sea_count.ensure(1));
        FRAC_TRY(up(c->d_sea_bend.ptr, ee.data(), ee.size() * sizeof(uint32_t)));
        size_t t1 = 0, t2 = 0;
        FRAC_HIP(c, sort_pairs_u32(nullptr, t1, c->d_sea_dkey.ptr, c->d_sea_dkey2.ptr, c->d_sea_dpos.ptr,
                                   c->d_sea_dpos2.ptr, P, 20, c->stream));
        FRAC_HIP(c, sort_pairs_u32(nullptr, t2, c->d_sea_rkey.ptr, c->d_sea_rkey2.ptr, c->d_sea_rord.ptr,
                                   c->d_sea_rord2.ptr, nr, 17, c->stream));
        size_t t3 = 0;
        FRAC_HIP(c, sort_pairs_u32(nullptr, t3, c->d_sea_rkey.ptr, c->d_sea_rkey2.ptr, c->d_sea_rord.ptr,
                                   c->d_sea_rord2.ptr, nr, 20, c->stream));
        c->sea_tmp_bytes = std::max<size_t>(std::max(std::max(t1, t2), t3), 1);
        FRAC_HIP(c, c->d_sea_tmp.ensure(c->sea_tmp_bytes));
    }
    if (c->tp) {
        const size_t ng = c->tp_groups.size(), nbk = c->nblocks, nt = c->ntiles;
        FRAC_HIP(c, c->d_m_slot_range.ensure(std::max<size_t>(nbk * 32, 1)));
        FRAC_HIP(c, c->d_m_range_slot.ensure(std::max<size_t>(nr, 1)));
        FRAC_HIP(c, c->d_m_tile_pos.ensure(std::max<size_t>(nt * 32, 1)));
        FRAC_HIP(c, c->d_m_dtiles.ensure(std::max<size_t>(nt * kTpKS * 64, 1)));
        FRAC_HIP(c, c->d_m_dconst.ensure((size_t)nt * kDftCS * 4 + 256)); // Fourier layout + one DMA piece of slack
        FRAC_HIP(c, c->d_m_rfrags.ensure(std::max<size_t>(nbk * 7 * 64, 1)));
        FRAC_HIP(c, c->d_m_rconst.ensure(std::max<size_t>(nbk * 32, 1)));
        FRAC_HIP(c, c->d_dft_tguard.ensure(std::max<size_t>(nt, 1)));
        FRAC_HIP(c, c->d_dft_tpool.ensure(std::max<size_t>(nt * 32 * 32, 1)));
        FRAC_HIP(c, c->d_dft_rguard.ensure(std::max<size_t>(nbk, 1)));
        FRAC_HIP(c, c->d_m8_work.ensure(std::max<size_t>(ng, 1)));
        FRAC_HIP(c, c->d_m8_blk_ptr.ensure(nbk + 1));
        FRAC_HIP(c, c->d_tp_groups.ensure(std::max<size_t>(ng, 1)));
        FRAC_HIP(c, c->d_tp_blk_group.ensure(std::max<size_t>(nbk, 1)));
        FRAC_HIP(c, c->d_tp_tile_sd.ensure(std::max<size_t>(nt, 1)));
        FRAC_HIP(c, c->d_tp_row_of.ensure(std::max<size_t>(P, 1)));
        FRAC_HIP(c, c->d_tp_blk_sr.ensure(std::max<size_t>(nbk, 1)));
        FRAC_HIP(c, c->d_tp_blk_u.ensure(std::max<size_t>(nbk, 1)));
        FRAC_HIP(c, c->d_tp_nch.ensure(ng + 1));
        FRAC_HIP(c, c->d_tp_choff.ensure(ng + 1));
        FRAC_HIP(c, c->d_tp_blkcnt.ensure(nbk + 1));
        FRAC_HIP(c, c->d_tp_tot.ensure(4));
        FRAC_HIP(c, c->d_tp_pairs.ensure(std::max<size_t>(ng, 1)));
        FRAC_HIP(c, c->d_tp_rbk.ensure(std::max<size_t>(nr, 1)));
        FRAC_TRY(up(c->d_tp_groups.ptr, c->tp_groups.data(), ng * sizeof(uint4)));
        FRAC_TRY(up(c->d_tp_blk_group.ptr, c->tp_blk_group.data(), nbk * sizeof(uint2)));
        if (nr)
            FRAC_HIP(c, hipMemcpyAsync(c->d_tp_rbk.ptr, c->d_rkey.ptr, nr * sizeof(int32_t), hipMemcpyDeviceToDevice,
                                       c->stream));
        c->tp_iota.resize(ng);
        for (size_t g = 0; g < ng; ++g)
            c->tp_iota[g] = (uint32_t)g;
        FRAC_HIP(c, c->d_tp_iota.ensure(std::max<size_t>(ng, 1)));
        FRAC_TRY(up(c->d_tp_iota.ptr, c->tp_iota.data(), ng * sizeof(uint32_t)));
        size_t s1 = 0, s2 = 0;
        FRAC_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, s1, c->d_tp_nch.ptr, c->d_tp_choff.ptr, (int)(ng + 1),
                                                     c->stream));
        FRAC_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, s2, c->d_tp_blkcnt.ptr, c->d_m8_blk_ptr.ptr,
                                                     (int)(nbk + 1), c->stream));
        c->tp_tmp_bytes = std::max<size_t>(std::max(s1, s2), 1);
        FRAC_HIP(c, c->d_tp_tmp.ensure(c->tp_tmp_bytes));
    }
    if (c->engine == FRAC_ENGINE_MFMA) {
        const int KS = (n * n + 15) / 16;
        // (T = 8 Fourier: the flipped copies' slots map to the same ranges, second half)
        FRAC_HIP(c, c->d_m_slot_range.ensure((size_t)c->nblocks * 32 * c->dft_copies));
        FRAC_HIP(c, c->d_m_range_slot.ensure(nr));
        FRAC_HIP(c, c->d_m_tile_pos.ensure((size_t)c->ntiles * 32));
        FRAC_HIP(c, c->d_m_work.ensure(c->m_work.size()));
        FRAC_HIP(c, c->d_m_blk_ptr.ensure(c->m_blk_ptr.size()));
        FRAC_HIP(c, c->d_m_blk_ent.ensure(c->m_blk_ent.size()));
        FRAC_HIP(c, c->d_m_rconst.ensure((size_t)c->nblocks * 32 * c->dft_copies));
        // the direct form's [tile][8] uint4 and the Fourier form's [tile][kDftCS] (+ one LDS-DMA piece of slack)
        FRAC_HIP(c, c->d_m_dconst.ensure((size_t)c->ntiles * kDftCS * 4 + 256));
        FRAC_HIP(c, c->d_m_dtiles.ensure((size_t)c->ntiles * KS * 64));
        FRAC_HIP(c, c->d_m_rfrags.ensure((size_t)c->nblocks * std::max(c->Teff * KS, 6u * c->dft_copies) * 64));
        FRAC_HIP(c, c->d_m_entries.ensure(std::max(c->m_work.size() * 4 * c->Teff, c->m8_work.size() * c->m8_bpw) *
                                          64));
        if (!c->m8_blk_ptr.empty()) { // built for n = 8, T = 4 (search_dft); may have no work
            FRAC_HIP(c, c->d_m8_work.ensure(std::max<size_t>(c->m8_work.size(), 1)));
            FRAC_HIP(c, c->d_m8_blk_ptr.ensure(c->m8_blk_ptr.size()));
            FRAC_HIP(c, c->d_m8_blk_ent.ensure(c->m8_blk_ent.size()));
            FRAC_TRY(up(c->d_m8_work.ptr, c->m8_work.data(), c->m8_work.size() * sizeof(uint4)));
            FRAC_TRY(up(c->d_m8_blk_ptr.ptr, c->m8_blk_ptr.data(), c->m8_blk_ptr.size() * sizeof(uint32_t)));
            FRAC_TRY(up(c->d_m8_blk_ent.ptr, c->m8_blk_ent.data(), c->m8_blk_ent.size() * sizeof(uint32_t)));
        }
        if (c->nblocks) {
            fill_range_slots<<<(c->nblocks * 32 + 255) / 256, 256, 0, c->stream>>>(
                c->mlayout, c->d_rord.ptr, c->nblocks * 32, c->d_m_slot_range.ptr, c->d_m_range_slot.ptr);
            if (c->dft_copies == 2)
                FRAC_HIP(c, hipMemcpyAsync(c->d_m_slot_range.ptr + (size_t)c->nblocks * 32, c->d_m_slot_range.ptr,
                                           (size_t)c->nblocks * 32 * sizeof(int32_t), hipMemcpyDeviceToDevice,
                                           c->stream));
        }
        if (c->ntiles)
            fill_tile_pos<<<(c->ntiles * 32 + 255) / 256, 256, 0, c->stream>>>(c->mlayout, c->ntiles * 32,
                                                                              c->d_m_tile_pos.ptr);
        FRAC_TRY(up(c->d_m_work.ptr, c->m_work.data(), c->m_work.size() * sizeof(uint4)));
        FRAC_TRY(up(c->d_m_blk_ptr.ptr, c->m_blk_ptr.data(), c->m_blk_ptr.size() * sizeof(uint32_t)));
        FRAC_TRY(up(c->d_m_blk_ent.ptr, c->m_blk_ent.data(), c->m_blk_ent.size() * sizeof(uint32_t)));
    }
    c->h_aux.resize(nr);
    c->dirty = false;
    tr.mark("uploads");
    return FRAC_OK;
}

template <int N, int T, int VAR>
void launch_search_mfma_v(frac_ctx* c, const MfmaSearchArgs& a)
{
    c->mfma_var_ran = VAR; // the resolve reads the entry layout this launch writes (VAR 128: merged over t)
    // H = 0 (the default threshold): a hit is S16 = 0, the smallest possible error, so
    // the plain first-minimum search already finds the first hit
    if (c->hitH > 0)
        search_mfma<N, T, true, VAR><<<a.nwork, 256, 0, c->stream>>>(a);
    else
        search_mfma<N, T, false, VAR><<<a.nwork, 256, 0, c->stream>>>(a);
}

// FRAC_MFMA_VARIANT (A/B knob, read per run): schedule variant of the MFMA searches. Every
// value a product build accepts gives identical (exact) records; the ablations, which give
// wrong results by design, are accepted — and compiled — only by a -DFRAC_TUNING build.
// Any other value fails the run (FRAC_E_INVALID), so a stray variable cannot corrupt records.
//   search_mfma: 0..7 schedule bits, 32 s_setprio, 64 late constants, 96, 98, 128 / 130 (default)
//                the minimum over transforms first; ablations 8, 16
//   search_dft:  default 8-wave exact form; 1 / 3 four-wave exact / guarded; 5 eight-tile
//                stages; 6 pairwise-tree row maximum; 12 two range blocks per wave (search_dft2);
//                ablations 9, 17, 41, 73, 105, 65 (four-wave) and 201..207 (eight-wave)
inline int mfma_variant(frac_ctx* c, int& var)
{
    const char* v = ab_knob("FRAC_MFMA_VARIANT");
    var = kDefaultMfmaVariant;
    if (!v || !*v)
        return FRAC_OK;
    char* end = nullptr;
    const long x = strtol(v, &end, 10);
    static const int exact[] = {0,  1,  2,  3,  4,  5,  6,  7,  12, 20, 21, 22, 23, 24, 26,
                                28, 27, 32, 33, 34, 35, 36, 64, 96, 98, 128, 130, 386};
    static const int ablation[] = {8, 9, 16, 17, 41, 65, 73, 105, 201, 202, 203, 204, 205, 206, 207, 226, 227, 240, 241, 242, 243};
    bool ok = end && *end == 0;
    bool known = false;
    for (int e : exact)
        known |= x == e;
    if (kTuningBuild)
        for (int e : ablation)
            known |= x == e;
    if (!ok || !known)
        return c->fail(FRAC_E_INVALID, std::string("FRAC_MFMA_VARIANT=") + v +
                                           (kTuningBuild ? " is unknown" : " is not a product variant (ablations need "
                                                                           "a -DFRAC_TUNING build)"));
    var = (int)x;
    return FRAC_OK;
}

// the direct form's schedule variant for range side N: the shipped one (the float-C epilogue for
// n ≤ 4, where it is exact), or in a tuning build FRAC_MFMA_VARIANT (386 falls back to 130 above n = 4)
template <int N>
int direct_variant(frac_ctx* c, int& var)
{
    FRAC_TRY(mfma_variant(c, var));
    const bool knob = kTuningBuild && ab_knob("FRAC_MFMA_VARIANT") && *ab_knob("FRAC_MFMA_VARIANT");
    if (!knob)
        var = N <= 4 ? kDefaultMfmaVariant4 : kDefaultMfmaVariant;
    if (N > 4 && (var & 256))
        var = kDefaultMfmaVariant;
    return FRAC_OK;
}

template <int N, int T>
int launch_search_mfma(frac_ctx* c, const MfmaSearchArgs& a)
{
    int var = 0;
    FRAC_TRY(direct_variant<N>(c, var));
#ifndef FRAC_TUNING
    (void)var; // the product build: the shipped schedule only
    launch_search_mfma_v<N, T, (N <= 4 ? kDefaultMfmaVariant4 : kDefaultMfmaVariant)>(c, a);
#else
    switch (var) {
    case 0: launch_search_mfma_v<N, T, 0>(c, a); break;
    case 1: launch_search_mfma_v<N, T, 1>(c, a); break;
    case 2: launch_search_mfma_v<N, T, 2>(c, a); break;
    case 3: launch_search_mfma_v<N, T, 3>(c, a); break;
    case 4: launch_search_mfma_v<N, T, 4>(c, a); break;
    case 5: launch_search_mfma_v<N, T, 5>(c, a); break;
    case 6: launch_search_mfma_v<N, T, 6>(c, a); break;
    case 7: launch_search_mfma_v<N, T, 7>(c, a); break;
    case 32: launch_search_mfma_v<N, T, 32>(c, a); break; // s_setprio around MFMA clusters
    case 64: launch_search_mfma_v<N, T, 64>(c, a); break; // late epilogue-constant reads
    case 96: launch_search_mfma_v<N, T, 96>(c, a); break;
    case 98: launch_search_mfma_v<N, T, 98>(c, a); break;
    case 128: launch_search_mfma_v<N, T, 128>(c, a); break; // minimum over transforms first
    case 130: launch_search_mfma_v<N, T, 130>(c, a); break;
    case 8: launch_search_mfma_v<N, T, 8>(c, a); break;   // ablation: 1-value epilogue
    case 16: launch_search_mfma_v<N, T, 16>(c, a); break; // ablation: no MFMA
    case 386:
        if constexpr (N <= 4) {
            launch_search_mfma_v<N, T, 386>(c, a); // the float-C epilogue
            break;
        }
        [[fallthrough]];
    default: launch_search_mfma_v<N, T, kDefaultMfmaVariant>(c, a); break;
    }
#endif
    return FRAC_OK;
}

// FRAC_FLAG_DIRECT_FORM (and, in a tuning build, FRAC_MFMA_DFT=0): the direct MFMA search for
// ratio-2 n = 8 instead of the rotation-group Fourier form (fracenc_dft.hip)
inline bool mfma_dft_enabled(const frac_ctx* c)
{
    if (c->p.flags & FRAC_FLAG_DIRECT_FORM)
        return false;
    const char* v = ab_knob("FRAC_MFMA_DFT");
    return v ? atoi(v) != 0 : true;
}

// whether launch_mfma<8> takes the Fourier path (launch_dft); launch_all leaves the run's
// best_key / fb_count resets to it then
inline bool dft_route(const frac_ctx* c)
{
    return (c->Teff == 4 || c->dft_copies == 2) && !c->virt && mfma_dft_enabled(c);
}

// The fit kernels' arguments for the current run (also carried by resolve_dft when it fuses the fit)
inline FitArgs fit_args(const frac_ctx* c, const uint8_t* dtgt, uint32_t tstride, uint32_t nr)
{
    FitArgs f;
    f.tgt = dtgt;
    f.tstride = tstride;
    f.ranges = c->d_ranges.ptr;
    f.doms = c->d_doms.ptr;
    f.porig = c->d_porig.ptr;
    f.pool = c->d_pool.ptr;
    f.best_key = c->d_best_key.ptr;
    f.nr = nr;
    f.T = c->p.transforms;
    f.hitH = c->hitH;
    f.smax = c->p.s_max;
    f.all_fallback = 0;
    f.out = c->d_out.ptr;
    f.aux = c->d_aux.ptr;
    f.fb_count = c->d_fb_count.ptr;
    f.fb_list = c->d_fb_list.ptr;
    f.plan = c->qplan;
    return f;
}

// fallback_grid's scratch at the list's capacity: kKeyNone / 0 when (re)allocated, kept so by the kernel
inline int ensure_fb_scratch(frac_ctx* c)
{
    const size_t n = std::max<size_t>(c->d_fb_list.cap, 1);
    if (c->d_fb_key.cap >= n && c->d_fb_done.cap >= n && c->d_fb_key.ptr && c->d_fb_done.ptr)
        return FRAC_OK;
    FRAC_HIP(c, c->d_fb_key.ensure(n));
    FRAC_HIP(c, c->d_fb_done.ensure(n));
    FRAC_HIP(c, hipMemsetAsync(c->d_fb_key.ptr, 0xff, c->d_fb_key.cap * sizeof(unsigned long long), c->stream));
    FRAC_HIP(c, hipMemsetAsync(c->d_fb_done.ptr, 0, c->d_fb_done.cap * sizeof(uint32_t), c->stream));
    return FRAC_OK;
}

// the fp32 fallback's arguments for the current run (fallback_grid)
inline FallbackArgs fallback_args(frac_ctx* c, const uint8_t* dtgt, uint32_t tstride)
{
    FallbackArgs b;
    b.tgt = dtgt;
    b.tstride = tstride;
    b.ranges = c->d_ranges.ptr;
    b.doms = c->d_doms.ptr;
    b.porig = c->d_porig.ptr;
    b.pool = c->d_pool.ptr;
    b.rbucket = c->d_rbucket.ptr;
    b.fb_count = c->d_fb_count.ptr;
    b.fb_list = c->d_fb_list.ptr;
    b.T = c->p.transforms;
    b.thr = c->p.rms_threshold;
    b.smax = c->p.s_max;
    b.out = c->d_out.ptr;
    b.aux = c->d_aux.ptr;
    b.tuples = c->fit_fused && !c->qplan ? c->tuple_sink : nullptr; // the fused resolvers' sink, if any
    b.fb_key = c->d_fb_key.ptr;
    b.fb_done = c->d_fb_done.ptr;
    // jobs per listed range: the largest bucket's domains in chunks of kFbChunk (a planned level: every domain)
    size_t maxb = 0;
    for (size_t k = 0; k < c->bucket_begin.size() && k < c->bucket_end.size(); ++k)
        maxb = std::max<size_t>(maxb, c->bucket_end[k] - c->bucket_begin[k]);
    if (c->qplan || maxb == 0)
        maxb = c->doms.size();
    b.chunks = (uint32_t)std::max<size_t>((maxb + kFbChunk - 1) / kFbChunk, 1);
    return b;
}

template <int N>
void launch_fallback_grid(frac_ctx* c, const FallbackArgs& b)
{
    fallback_grid<N><<<kFallbackBlocks, 256, 0, c->stream>>>(b);
}

// The fused resolvers' listed fp32-regime ranges, settled before anything reads the run's records: one
// fallback_grid launch (an empty list costs its dispatch).  frac_fetch settles only when a range was listed.
inline int settle_fallback(frac_ctx* c)
{
    if (!c->fb_pending)
        return FRAC_OK;
    c->fb_pending = false;
    if (c->fb_n == 16)
        launch_fallback_grid<16>(c, c->fb_args);
    else
        launch_fallback_grid<8>(c, c->fb_args);
    FRAC_HIP(c, hipGetLastError());
    return FRAC_OK;
}

// work items a search launch covers: the host-built list, or a device-planned level's bound (its
// workgroups past DevPlan::nwork leave at once)
inline uint32_t launch_nwork(const frac_ctx* c, const std::vector<uint4>& w)
{
    return c->qplan ? c->qp_nwork_cap : (uint32_t)w.size();
}

#ifdef FRAC_CLOCK_STAMP
// the diagnostic clock build (tools/build_tuning.py --stamps): search_dft stamps s_memtime and
// s_memrealtime around its loop, per workgroup, into this buffer; frac_clock_stamps reads the last
// launch's.  Never in the product or the plain tuning build.
static unsigned long long* g_stamps = nullptr;
static size_t g_stamps_cap = 0;
static unsigned g_stamps_n = 0;
static unsigned long long* clock_stamps_for(unsigned nwg)
{
    if (nwg > g_stamps_cap) {
        if (g_stamps)
            (void)hipFree(g_stamps);
        g_stamps = nullptr;
        g_stamps_cap = 0;
        if (hipMalloc(&g_stamps, (size_t)nwg * kClockStampWords * sizeof(unsigned long long)) != hipSuccess)
            return nullptr;
        g_stamps_cap = nwg;
    }
    g_stamps_n = nwg;
    return g_stamps;
}
// out: [cap_workgroups][kClockStampWords]
extern "C" int frac_clock_stamps(unsigned long long* out, size_t cap_workgroups)
{
    if (!g_stamps || !out)
        return -1;
    const size_t n = std::min<size_t>(g_stamps_n, cap_workgroups);
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(out, g_stamps, n * kClockStampWords * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return (int)n;
}
#endif

// n = 8, T = 4: the C4-Fourier search (6 MFMAs per 32×32 tile pair instead of 16).  inits: reset
// best_key and fb_count in the preparation kernel (launch_all skipped its memsets)
inline int launch_dft(frac_ctx* c, const uint8_t* dtgt, uint32_t tstride, bool inits)
{
    const uint32_t nr = (uint32_t)nranges(c);
    MfmaDomainPrepArgs d;
    d.pool = c->d_pool.ptr;
    d.negsd2 = c->d_negsd2.ptr;
    d.tile_pos = c->d_m_tile_pos.ptr;
    d.ntiles = c->ntiles;
    d.dtiles = c->d_m_dtiles.ptr;
    d.dconst = c->d_m_dconst.ptr;
    d.plan = c->qplan;
    FRAC_HIP(c, c->d_dft_tguard.ensure(std::max<size_t>(c->ntiles, 1)));
    FRAC_HIP(c, c->d_dft_trmax.ensure((size_t)c->ntiles + 4)); // + 4: a chunk's thresholds are one scalar load
    FRAC_HIP(c, c->d_dft_tpool.ensure(std::max<size_t>((size_t)c->ntiles * 32 * 32, 1)));
    const uint32_t nbk = c->nblocks * c->dft_copies; // range blocks incl. T = 8's flipped copies
    FRAC_HIP(c, c->d_dft_rguard.ensure(std::max<size_t>(nbk, 1)));
    // FRAC_MFMA_VARIANT for this path (A/B knob): default = exact form in 8-wave workgroups
    // with the v_max3-chain row maximum; 20 = the five-MFMA form (kDft5) in the same
    // workgroups; 6 = the pairwise-tree row maximum; 5 = 8-tile stages; 12 = two range blocks
    // per wave; 1 = exact form in 4-wave workgroups, 3 = guarded fast path (4 waves), odd
    // values ≥ 9 = ablations of variant 1 (tuning only: wrong results)
    int var = 0;
    FRAC_TRY(mfma_variant(c, var));
    var = dft_variant(var);
    const int form = dft_form(var);
    const bool f5 = form != 4; // five domain fragments per tile (forms 5 and 6)
    FRAC_HIP(c, c->d_m_dtiles.ensure(std::max<size_t>((size_t)c->ntiles * (f5 ? 5 : 4) * 64, 1)));
    d.dtiles = c->d_m_dtiles.ptr;
    DftDomainBuildArgs b;
    b.src = c->d_src.ptr;
    b.sstride = c->d_sstride;
    b.doms = c->d_doms.ptr;
    b.porig = c->d_porig.ptr;
    b.pool = c->d_pool.ptr;
    b.negsd2 = c->d_negsd2.ptr;
    b.tpool = c->d_dft_tpool.ptr;
    MfmaRangePrepArgs r;
    r.tgt = dtgt;
    r.tstride = tstride;
    r.ranges = c->d_ranges.ptr;
    r.slot_range = c->d_m_slot_range.ptr;
    r.nblocks = nbk;
    r.T = 4;
    r.rfrags = c->d_m_rfrags.ptr;
    r.rconst = c->d_m_rconst.ptr;
    r.flip_from = c->dft_copies == 2 ? c->nblocks : ~0u;
    r.plan = c->qplan;
    FRAC_HIP(c, c->d_dft_rorb.ensure(std::max<size_t>((size_t)r.nblocks * 32 * 32, 1)));
    r.rorb = c->d_dft_rorb.ptr;
    // the search merges its domain splits per slot (64-bit atomicMax; reset by the range prep), so the resolve
    // reads one word per slot instead of walking the block's entries through the CSR map
    // (search_dft2, an A/B form of the tuning build, writes entries only)
    const bool slotbest = !(kTuningBuild && ((form == 6 && var == 23) || (!dft_four_wave(var) && var == 12)));
    FRAC_HIP(c, c->d_dft_slotbest.ensure(std::max<size_t>((size_t)r.nblocks * 32, 1)));
    r.slotbest = slotbest ? c->d_dft_slotbest.ptr : nullptr;
    // one launch: domain tiles, range blocks and (inits) the run's resets
    DftPrepInit in;
    if (inits) {
        in.best_key = c->d_best_key.ptr;
        in.nr = nr;
        in.fb_count = c->d_fb_count.ptr;
        in.fbc = 0; // the Fourier path never runs with all_fallback
    }
    in.dblocks = (c->ntiles * 64 + 255) / 256; // two lanes per tile row (dft_domain_build_pair_at)
    in.plan = c->qplan;
    in.copies = c->dft_copies;
    const unsigned pg = in.dblocks + (nbk * 64 + 255) / 256; // two lanes per range slot (dft_range_prep_pair_at)
    if (pg || inits) {
        int32_t* trmax = f5 ? c->d_dft_trmax.ptr : nullptr;
        const dim3 grid(std::max(pg, 1u));
        if (form == 5)
            dft_prep<5><<<grid, 256, 0, c->stream>>>(d, b, c->d_dft_tguard.ptr, trmax, r, c->d_dft_rguard.ptr, in);
        else if (form == 6)
            dft_prep<6><<<grid, 256, 0, c->stream>>>(d, b, c->d_dft_tguard.ptr, trmax, r, c->d_dft_rguard.ptr, in);
        else
            dft_prep<4><<<grid, 256, 0, c->stream>>>(d, b, c->d_dft_tguard.ptr, trmax, r, c->d_dft_rguard.ptr, in);
    }
    if (c->p.flags & FRAC_FLAG_TIMING)
        FRAC_TRY(mark_event(c, 1));
    const bool four = dft_four_wave(var);
    const std::vector<uint4>& work = four ? c->m_work : c->m8_work;
    c->form_ran = FRAC_FORM_FOURIER;
    c->flops_ran = 0;
    for (const uint4& w : work) // 8 (forms 5 / 6: 5 / 6) MFMA 32x32x16 (32768 flops each) per (block, tile)
        c->flops_ran += (uint64_t)w.y * (w.w - w.z) * (form == 5 ? 5ull : form == 6 ? 6ull : 8ull) * 32768ull;
    const uint32_t nwork = launch_nwork(c, work);
    if (nwork) {
        MfmaSearchArgs a;
        a.dtiles = c->d_m_dtiles.ptr;
        a.dconst = reinterpret_cast<const uint4*>(c->d_m_dconst.ptr);
        a.rfrags = c->d_m_rfrags.ptr;
        a.rconst = c->d_m_rconst.ptr;
        a.work = four ? c->d_m_work.ptr : c->d_m8_work.ptr;
        a.nwork = nwork;
        a.hitH = (uint32_t)std::max<int64_t>(c->hitH, 0);
        a.entries = c->d_m_entries.ptr;
        a.plan = c->qplan;
        DftArgs da;
        da.m = a;
        da.rguard = c->d_dft_rguard.ptr;
        da.tguard = c->d_dft_tguard.ptr;
        da.trmax = c->d_dft_trmax.ptr;
        da.slotbest = r.slotbest;
        const unsigned nwg = nwork;
#ifdef FRAC_CLOCK_STAMP
        da.stamps = clock_stamps_for(nwg);
#endif
        const bool hits = c->hitH > 0;
        constexpr uint32_t W8 = kDftBlocksPerWG;
#ifndef FRAC_TUNING
        // the product build: the shipped form only (variant 35, kDftDefaultVariant) — the six-MFMA
        // form with the guarded constant-folded epilogue, the unrolled chunk and buffer_load … lds stages
        static_assert(kDftDefaultVariant == 35, "the product build's Fourier search is variant 35");
        (void)four;
        constexpr int V35 = 1 | kDftChain | kDft6 | kDftFast6 | kDftUnroll | kDftBufDma;
        // few tiles: the run is a short chain whose resolve weighs as much as its search, and the search also
        // carries the tiles of the winning chunk that attain its maximum (TMASK) so the resolve evaluates those
        if (c->ntiles <= kDftTmaskTiles) {
            if (hits)
                search_dft<true, V35, W8, kTilesPerStage, false, true><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, V35, W8, kTilesPerStage, false, true><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (hits) {
            search_dft<true, V35, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else {
            search_dft<false, V35, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        }
#else // the tuning build: every A/B variant and ablation
        if (form == 6 && var == 37) { // variant 35 carrying the winning chunk's tile mask (TMASK)
            constexpr int V35 = 1 | kDftChain | kDft6 | kDftFast6 | kDftUnroll | kDftBufDma;
            if (hits)
                search_dft<true, V35, W8, kTilesPerStage, false, true><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, V35, W8, kTilesPerStage, false, true><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (!four && var >= 200) {
            // ablations of the 8-wave exact form (wrong results by design)
            switch (var) {
            case 201: search_dft<false, 9, W8><<<nwg, 64 * W8, 0, c->stream>>>(da); break;   // MFMA-only
            case 202: search_dft<false, 73, W8><<<nwg, 64 * W8, 0, c->stream>>>(da); break;  // MFMA-only, no DMA/bar
            case 203: search_dft<false, 265, W8><<<nwg, 64 * W8, 0, c->stream>>>(da); break; // MFMA-only, no DMA
            case 204: search_dft<false, 521, W8><<<nwg, 64 * W8, 0, c->stream>>>(da); break; // MFMA-only, no barrier
            case 205: search_dft<false, 257, W8><<<nwg, 64 * W8, 0, c->stream>>>(da); break; // full, no DMA
            case 206: search_dft<false, 513, W8><<<nwg, 64 * W8, 0, c->stream>>>(da); break; // full, no barrier
            case 226: // the guarded six-MFMA form (26), no barrier
                search_dft<false, 1 | kDftChain | kDft6 | kDftFast6 | 512, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                break;
            case 227: // the guarded six-MFMA form (26), no LDS-DMA / barrier after the first stages
                search_dft<false, 1 | kDftChain | kDft6 | kDftFast6 | 64, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                break;
            case 240: // variant 35, MFMAs with a one-value epilogue
                search_dft<false, 1 | kDftChain | kDft6 | kDftFast6 | kDftUnroll | kDftBufDma | 8, W8><<<nwg, 64 * W8, 0,
                                                                                                    c->stream>>>(da);
                break;
            case 241: // variant 35, the fast epilogue without MFMAs
                search_dft<false, 1 | kDftChain | kDft6 | kDftFast6 | kDftUnroll | kDftBufDma | 16, W8><<<nwg, 64 * W8, 0,
                                                                                                     c->stream>>>(da);
                break;
            case 242: // variant 35, no barrier
                search_dft<false, 1 | kDftChain | kDft6 | kDftFast6 | kDftUnroll | kDftBufDma | 512, W8><<<nwg, 64 * W8,
                                                                                                      0, c->stream>>>(da);
                break;
            case 243: // variant 35, no LDS-DMA / barrier after the first stages
                search_dft<false, 1 | kDftChain | kDft6 | kDftFast6 | kDftUnroll | kDftBufDma | 64, W8><<<nwg, 64 * W8, 0,
                                                                                                     c->stream>>>(da);
                break;
            default: search_dft<false, 65, W8><<<nwg, 64 * W8, 0, c->stream>>>(da); break;  // full, no DMA/bar
            }
        } else if (form == 6 && var == 23) { // the six-MFMA form, two range blocks per wave (search_dft2)
            if (hits)
                search_dft2<true, true><<<nwg, 256, 0, c->stream>>>(da);
            else
                search_dft2<false, true><<<nwg, 256, 0, c->stream>>>(da);
        } else if (form == 6 && (var == 27 || var == 28)) { // 16 range blocks per (1024-thread) workgroup
            if (c->m8_bpw != 16)
                return c->fail(FRAC_E_STATE, "search_dft: work lists built for another workgroup size");
            if (var == 27) {
                if (hits)
                    search_dft<true, 1 | kDftChain | kDft6, 16><<<nwg, 1024, 0, c->stream>>>(da);
                else
                    search_dft<false, 1 | kDftChain | kDft6, 16><<<nwg, 1024, 0, c->stream>>>(da);
            } else {
                if (hits)
                    search_dft<true, 1 | kDftChain | kDft6 | kDftFast6, 16><<<nwg, 1024, 0, c->stream>>>(da);
                else
                    search_dft<false, 1 | kDftChain | kDft6 | kDftFast6, 16><<<nwg, 1024, 0, c->stream>>>(da);
            }
        } else if (form == 6 && var >= 33 && var <= 36) { // 26 with the issue-cost knobs
            constexpr int V = 1 | kDftChain | kDft6 | kDftFast6;
            switch (var) {
            case 33: // unrolled chunk
                if (hits)
                    search_dft<true, V | kDftUnroll, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                else
                    search_dft<false, V | kDftUnroll, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                break;
            case 34: // buffer_load … lds stages
                if (hits)
                    search_dft<true, V | kDftBufDma, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                else
                    search_dft<false, V | kDftBufDma, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                break;
            case 35: // both
                if (hits)
                    search_dft<true, V | kDftUnroll | kDftBufDma, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                else
                    search_dft<false, V | kDftUnroll | kDftBufDma, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                break;
            default: // both, second half of the waves at s_setprio 1
                if (hits)
                    search_dft<true, V | kDftUnroll | kDftBufDma | kDftPrio, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                else
                    search_dft<false, V | kDftUnroll | kDftBufDma | kDftPrio, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
                break;
            }
        } else if (form == 6 && var == 26) { // the six-MFMA form, guarded constant-folded epilogue
            if (hits)
                search_dft<true, 1 | kDftChain | kDft6 | kDftFast6, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, 1 | kDftChain | kDft6 | kDftFast6, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (form == 6) { // the six-MFMA form
            if (hits)
                search_dft<true, 1 | kDftChain | kDft6, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, 1 | kDftChain | kDft6, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (var == 22) { // the five-MFMA form, unpacked epilogue
            if (hits)
                search_dft<true, 1 | kDftChain | kDft5 | kDftScalar, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, 1 | kDftChain | kDft5 | kDftScalar, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (form == 5) { // the five-MFMA form
            if (hits)
                search_dft<true, 1 | kDftChain | kDft5, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, 1 | kDftChain | kDft5, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (!four && var == 5) { // 8-tile LDS stages
            if (hits)
                search_dft<true, 1 | kDftChain, W8, 8><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, 1 | kDftChain, W8, 8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (!four && var == 12) { // two range blocks per wave (4-wave workgroups, the 8-block lists)
            static_assert(kDftBlocksPerWG == 8, "search_dft2 covers 8 blocks per workgroup");
            if (hits)
                search_dft2<true><<<nwg, 256, 0, c->stream>>>(da);
            else
                search_dft2<false><<<nwg, 256, 0, c->stream>>>(da);
        } else if (!four && var == 6) { // the pairwise-tree row maximum (round 1's default, A/B)
            if (hits)
                search_dft<true, 1, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, 1, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (!four) {
            if (hits)
                search_dft<true, 1 | kDftChain, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
            else
                search_dft<false, 1 | kDftChain, W8><<<nwg, 64 * W8, 0, c->stream>>>(da);
        } else if (var == 1) {
            if (hits)
                search_dft<true, 1><<<nwg, 256, 0, c->stream>>>(da);
            else
                search_dft<false, 1><<<nwg, 256, 0, c->stream>>>(da);
        } else if (var == 3) {
            if (hits)
                search_dft<true, 0><<<nwg, 256, 0, c->stream>>>(da);
            else
                search_dft<false, 0><<<nwg, 256, 0, c->stream>>>(da);
        } else {
            // ablations of the 4-wave exact form (wrong results by design)
            switch (var) {
            case 9: search_dft<false, 9><<<nwg, 256, 0, c->stream>>>(da); break;     // MFMA-only
            case 17: search_dft<false, 17><<<nwg, 256, 0, c->stream>>>(da); break;   // VALU-only
            case 41: search_dft<false, 41><<<nwg, 256, 0, c->stream>>>(da); break;   // MFMA-only, no LDS reads
            case 73: search_dft<false, 73><<<nwg, 256, 0, c->stream>>>(da); break;   // MFMA-only, no DMA/barrier
            case 105: search_dft<false, 105><<<nwg, 256, 0, c->stream>>>(da); break; // MFMA-only, neither
            case 65: search_dft<false, 65><<<nwg, 256, 0, c->stream>>>(da); break;   // full, no DMA/barrier
            default: search_dft<false, 1><<<nwg, 256, 0, c->stream>>>(da); break;
            }
        }
#endif
    }
    if (c->p.flags & FRAC_FLAG_TIMING)
        FRAC_TRY(mark_event(c, 2));
    if (nr) {
        MfmaResolveArgs v;
        v.tgt = dtgt;
        v.tstride = tstride;
        v.ranges = c->d_ranges.ptr;
        v.range_slot = c->d_m_range_slot.ptr;
        v.blk_ptr = four ? c->d_m_blk_ptr.ptr : c->d_m8_blk_ptr.ptr;
        v.blk_ent = four ? c->d_m_blk_ent.ptr : c->d_m8_blk_ent.ptr;
        v.entries = c->d_m_entries.ptr;
        v.rconst = c->d_m_rconst.ptr;
        v.tile_pos = c->d_m_tile_pos.ptr;
        v.ntiles = c->ntiles;
        v.pool = c->d_pool.ptr;
        v.negsd2 = c->d_negsd2.ptr;
        v.nr = nr;
        v.T = c->dft_copies == 2 ? 8u : 4u;
        v.hitH = c->hitH;
        v.best_key = c->d_best_key.ptr;
        v.slot_range = c->d_m_slot_range.ptr;
        v.nslots = c->nblocks * 32u;
        v.flip_slots = c->dft_copies == 2 ? c->nblocks * 32u : 0u;
        v.tpool = c->d_dft_tpool.ptr;
        v.rorb = c->d_dft_rorb.ptr;
        v.slotbest = r.slotbest;
        v.plan = c->qplan;
        FRAC_HIP(c, c->d_rstat.ensure(std::max<size_t>(nr, 1)));
        v.rstat = c->d_rstat.ptr;
        v.fused_fit = 1; // the fit in the resolving wave (launch_all skips fit_rstat)
        v.fit = fit_args(c, dtgt, tstride, nr);
        v.fit.tuples = c->qplan ? nullptr : c->tuple_sink;
        c->fit_fused = true;
        // one-wave workgroups: a finished range frees its slot at once (0.254 vs 0.271 ms finish
        // against 4-wave workgroups, 30-sample A/B, profiles/r01/ab_fourier_variants.log); T = 8: two
        // waves, the slot and its flipped copy resolved at the same time
        v.paired = c->dft_copies == 2 ? 1 : 0;
        resolve_dft<false><<<std::max(1u, v.nslots), v.paired ? 128 : 64, 0, c->stream>>>(v);
    }
    return FRAC_OK;
}

template <int N>
int launch_mfma(frac_ctx* c, const uint8_t* dtgt, uint32_t tstride, bool inits = false)
{
    // T = the transforms per pool row: 1 in the sampled form (one row per domain and transform)
    const uint32_t nr = (uint32_t)nranges(c), T = c->Teff;
    if constexpr (N == 8) {
        if (dft_route(c))
            return launch_dft(c, dtgt, tstride, inits);
    }
    int dvar = 0;
    FRAC_TRY(direct_variant<N>(c, dvar));
    const int fmode = (dvar & 256) ? 1 : 0; // the float-C epilogue: its row constants and B scaling
    // n ≤ 4 with the transforms merged in the search (resolve_small): the search merges its work items per range
    // slot itself (one 64-bit atomicMax per slot and work item; reset by mfma_range_prep), so the resolve reads one
    // word per slot instead of walking the block's entries through the CSR map
    unsigned long long* slotbest = nullptr;
    if (N <= 4 && T >= 4 && (dvar & (128 | 256)) && c->nblocks) {
        FRAC_HIP(c, c->d_dft_slotbest.ensure((size_t)c->nblocks * 32));
        slotbest = c->d_dft_slotbest.ptr;
    }
    // the domain tiles and the range blocks' fragments in one launch (mfma_prep)
    MfmaDomainPrepArgs d;
    d.fmode = fmode;
    d.pool = c->d_pool.ptr;
    d.negsd2 = c->d_negsd2.ptr;
    d.tile_pos = c->d_m_tile_pos.ptr;
    d.ntiles = c->ntiles;
    d.dtiles = c->d_m_dtiles.ptr;
    d.dconst = c->d_m_dconst.ptr;
    d.plan = c->qplan;
    if ((N == 4 || N == 16) && !c->virt) { // the pool rows built here (launch_all skips pool_build)
        d.src = c->d_src.ptr;
        d.sstride = c->d_sstride;
        d.doms = c->d_doms.ptr;
        d.porig = c->d_porig.ptr;
        d.pool_out = c->d_pool.ptr;
        d.negsd2_out = c->d_negsd2.ptr;
    }
    MfmaRangePrepArgs r;
    r.tgt = dtgt;
    r.tstride = tstride;
    r.ranges = c->d_ranges.ptr;
    r.slot_range = c->d_m_slot_range.ptr;
    r.nblocks = c->nblocks;
    r.T = T;
    r.rfrags = c->d_m_rfrags.ptr;
    r.rconst = c->d_m_rconst.ptr;
    r.plan = c->qplan;
    r.fmode = fmode;
    r.slotbest = slotbest;
    // n = 16: 16 lanes per tile row and one workgroup per range block; else a thread per tile row and per
    // (block, transform, K-step, lane)
    const uint32_t dblocks = !c->ntiles ? 0u
                             : N == 16  ? (c->ntiles * 32 * MfmaGeom<16>::KS + 255) / 256
                                        : (c->ntiles * 32 + 255) / 256;
    const uint32_t rblocks = !c->nblocks ? 0u
                             : N == 16   ? c->nblocks
                                         : (uint32_t)(((size_t)c->nblocks * T * MfmaGeom<N>::KS * 64 + 255) / 256);
    // rconst is a sum of per-pixel terms, accumulated by the transform-0 threads (n < 16; a planned level's
    // qt_fill_maps zeroed it)
    if (N != 16 && c->nblocks && !c->qplan)
        FRAC_HIP(c, hipMemsetAsync(c->d_m_rconst.ptr, 0, (size_t)c->nblocks * 32 * sizeof(uint32_t), c->stream));
    if (dblocks + rblocks) {
        if constexpr (N == 16) {
            if (T == 8)
                mfma_prep<16, 8><<<dblocks + rblocks, 256, 0, c->stream>>>(d, r, dblocks);
            else if (T == 1)
                mfma_prep<16, 1><<<dblocks + rblocks, 256, 0, c->stream>>>(d, r, dblocks);
            else
                mfma_prep<16, 4><<<dblocks + rblocks, 256, 0, c->stream>>>(d, r, dblocks);
        } else {
            mfma_prep<N><<<dblocks + rblocks, 256, 0, c->stream>>>(d, r, dblocks);
        }
    }
    if (c->p.flags & FRAC_FLAG_TIMING)
        FRAC_TRY(mark_event(c, 1));
    c->form_ran = FRAC_FORM_DIRECT;
    c->flops_ran = 0;
    for (const uint4& w : c->m_work) // T·KS MFMA 32x32x16 per (range block, domain tile)
        c->flops_ran += (uint64_t)w.y * (w.w - w.z) * T * MfmaGeom<N>::KS * 32768ull;
    const uint32_t nwork = launch_nwork(c, c->m_work);
    if (nwork) {
        MfmaSearchArgs a;
        a.dtiles = c->d_m_dtiles.ptr;
        a.dconst = reinterpret_cast<const uint4*>(c->d_m_dconst.ptr);
        a.rfrags = c->d_m_rfrags.ptr;
        a.rconst = c->d_m_rconst.ptr;
        a.work = c->d_m_work.ptr;
        a.nwork = nwork;
        a.hitH = (uint32_t)std::max<int64_t>(c->hitH, 0);
        a.entries = c->d_m_entries.ptr;
        a.plan = c->qplan;
        a.slotbest = slotbest;
        if constexpr (N == 16) { // 4-wave workgroups: mfma16_bpw(T) range blocks × their T transforms
            const unsigned nwg = nwork;
            const bool hits = c->hitH > 0;
            if (T == 8) {
                if (hits)
                    search_mfma16<8, true><<<nwg, 256, 0, c->stream>>>(a);
                else
                    search_mfma16<8, false><<<nwg, 256, 0, c->stream>>>(a);
            } else if (T == 1) {
                if (hits)
                    search_mfma16<1, true><<<nwg, 256, 0, c->stream>>>(a);
                else
                    search_mfma16<1, false><<<nwg, 256, 0, c->stream>>>(a);
            } else {
                if (hits)
                    search_mfma16<4, true><<<nwg, 256, 0, c->stream>>>(a);
                else
                    search_mfma16<4, false><<<nwg, 256, 0, c->stream>>>(a);
            }
        } else if (T == 8)
            FRAC_TRY((launch_search_mfma<N, 8>(c, a)));
        else if (T == 1)
            FRAC_TRY((launch_search_mfma<N, 1>(c, a)));
        else
            FRAC_TRY((launch_search_mfma<N, 4>(c, a)));
    }
    if (c->p.flags & FRAC_FLAG_TIMING)
        FRAC_TRY(mark_event(c, 2));
    if (nr) {
        MfmaResolveArgs v;
        v.tgt = dtgt;
        v.tstride = tstride;
        v.ranges = c->d_ranges.ptr;
        v.range_slot = c->d_m_range_slot.ptr;
        v.blk_ptr = c->d_m_blk_ptr.ptr;
        v.blk_ent = c->d_m_blk_ent.ptr;
        v.entries = c->d_m_entries.ptr;
        v.rconst = c->d_m_rconst.ptr;
        v.tile_pos = c->d_m_tile_pos.ptr;
        v.ntiles = c->ntiles;
        v.pool = c->d_pool.ptr;
        v.negsd2 = c->d_negsd2.ptr;
        v.nr = nr;
        v.T = T;
        v.hitH = c->hitH;
        v.best_key = c->d_best_key.ptr;
        v.merged = (N != 16 && T > 1 && (c->mfma_var_ran & (128 | 256))) ? 1 : 0; // entries merged over t
        v.fmode = (N != 16 && (c->mfma_var_ran & 256)) ? 1 : 0;                  // fmap'd float-C minima
        v.slotbest = slotbest;
        if constexpr (N == 16)
            v.rfrags = c->d_m_rfrags.ptr; // the range copies from search_mfma16's B fragments
        if (!c->virt) { // the fit in the resolving wave (the sampled form fits at its own points: gen_fit)
            v.fused_fit = 1;
            v.fit = fit_args(c, dtgt, tstride, nr);
            v.fit.tuples = c->qplan ? nullptr : c->tuple_sink;
            c->fit_fused = true;
        }
        v.plan = c->qplan;
        if constexpr (N <= 4) {
            if (T >= 4) // a pool row per lane, the transforms across lanes
                resolve_small<N><<<(nr + 3) / 4, 256, 0, c->stream>>>(v);
            else
                resolve_mfma<N><<<(nr + 3) / 4, 256, 0, c->stream>>>(v);
        } else {
            resolve_mfma<N><<<(nr + 3) / 4, 256, 0, c->stream>>>(v);
        }
    }
    return FRAC_OK;
}

// SEA engine, tiled form (fracenc_tp.hip): sorted tiles and blocks, per-range seed bounds,
// per-group windows, the Fourier search over the windows with per-chunk entries, resolve_dft.
// One host synchronisation sizes the entry arrays (their count depends on the windows).
int launch_tp(frac_ctx* c, const uint8_t* dtgt, uint32_t tstride, bool timing)
{
    const uint32_t nr = (uint32_t)nranges(c), P = c->npos;
    const uint32_t nt = c->ntiles, nbk = c->nblocks, ng = (uint32_t)c->tp_groups.size();
    // resolve_dft<true> keeps one copy per slot: T = 8's flipped copies would go unmerged here, and
    // prepare() routes only T = 4 to the tiled form (c->tp)
    if (c->p.transforms != 4)
        return c->fail(FRAC_E_STATE, "the tiled SEA form runs T = 4 only");
    c->form_ran = FRAC_FORM_SEA_MFMA;
    c->flops_ran = 0;
    c->evaluated_ran = 0;
    if (P) {
        tp_domain_keys<<<(P + 255) / 256, 256, 0, c->stream>>>(c->d_src.ptr, c->d_sstride, c->d_doms.ptr,
                                                               c->d_porig.ptr, P, c->d_sea_bend.ptr,
                                                               (uint32_t)c->bucket_end.size(), c->d_sea_dkey.ptr,
                                                               c->d_sea_dpos.ptr);
        size_t tb = c->sea_tmp_bytes;
        FRAC_HIP(c, sort_pairs_u32(c->d_sea_tmp.ptr, tb, c->d_sea_dkey.ptr, c->d_sea_dkey2.ptr, c->d_sea_dpos.ptr,
                                   c->d_sea_dpos2.ptr, P, c->tp_key_bits, c->stream));
    }
    if (nt) {
        tp_build_tiles<<<(nt * 32 + 255) / 256, 256, 0, c->stream>>>(
            c->tp_bk, c->d_sea_dkey2.ptr, c->d_sea_dpos2.ptr, nt, c->d_m_tile_pos.ptr, c->d_tp_tile_sd.ptr,
            c->d_tp_row_of.ptr, c->d_m_dtiles.ptr, c->d_m_dconst.ptr, c->d_dft_tguard.ptr, kTpKS);
        MfmaDomainPrepArgs d;
        d.pool = c->d_pool.ptr;
        d.negsd2 = c->d_negsd2.ptr;
        d.tile_pos = c->d_m_tile_pos.ptr;
        d.ntiles = nt;
        d.dtiles = c->d_m_dtiles.ptr;
        d.dconst = c->d_m_dconst.ptr;
        DftDomainBuildArgs b;
        b.src = c->d_src.ptr;
        b.sstride = c->d_sstride;
        b.doms = c->d_doms.ptr;
        b.porig = c->d_porig.ptr;
        b.pool = c->d_pool.ptr;
        b.negsd2 = c->d_negsd2.ptr;
        b.tpool = c->d_dft_tpool.ptr;
        b.row_of = c->d_tp_row_of.ptr;
        b.npos = P;
        if (P)
            dft_domain_build<true, kDftTpForm != 4><<<(P + 255) / 256, 256, 0, c->stream>>>(d, b, c->d_dft_tguard.ptr);
    }
    if (nr) {
        tp_range_keys<<<(nr + 255) / 256, 256, 0, c->stream>>>(dtgt, tstride, c->d_ranges.ptr, c->d_tp_rbk.ptr, nr,
                                                               c->d_sea_rkey.ptr, c->d_sea_rord.ptr);
        size_t tb = c->sea_tmp_bytes;
        FRAC_HIP(c, sort_pairs_u32(c->d_sea_tmp.ptr, tb, c->d_sea_rkey.ptr, c->d_sea_rkey2.ptr, c->d_sea_rord.ptr,
                                   c->d_sea_rord2.ptr, nr, c->tp_key_bits, c->stream));
    }
    if (nbk) {
        tp_build_slots<<<(nbk * 32 + 255) / 256, 256, 0, c->stream>>>(c->tp_bk, c->d_sea_rkey2.ptr, c->d_sea_rord2.ptr,
                                                                      nbk, c->d_m_slot_range.ptr,
                                                                      c->d_m_range_slot.ptr, c->d_tp_blk_sr.ptr,
                                                                      c->d_tp_blk_u.ptr);
        MfmaRangePrepArgs r;
        r.tgt = dtgt;
        r.tstride = tstride;
        r.ranges = c->d_ranges.ptr;
        r.slot_range = c->d_m_slot_range.ptr;
        r.nblocks = nbk;
        r.T = 4;
        r.rfrags = c->d_m_rfrags.ptr;
        r.rconst = c->d_m_rconst.ptr;
        FRAC_HIP(c, c->d_dft_rorb.ensure(std::max<size_t>((size_t)r.nblocks * 32 * 32, 1)));
        r.rorb = c->d_dft_rorb.ptr;
        dft_range_prep<kDftTpForm><<<(nbk * 32 + 255) / 256, 256, 0, c->stream>>>(r, c->d_dft_rguard.ptr);
    }
    if (timing)
        FRAC_TRY(mark_event(c, 1));
    if (!nr || !ng) // no ranges, or no domain in any range's bucket: every record is the default
        return FRAC_OK;
    constexpr uint32_t W8 = kDftBlocksPerWG;
    MfmaSearchArgs a;
    a.dtiles = c->d_m_dtiles.ptr;
    a.dconst = reinterpret_cast<const uint4*>(c->d_m_dconst.ptr);
    a.rfrags = c->d_m_rfrags.ptr;
    a.rconst = c->d_m_rconst.ptr;
    a.work = c->d_m8_work.ptr;
    a.nwork = ng;
    a.hitH = (uint32_t)std::max<int64_t>(c->hitH, 0);
    a.entries = c->d_m_entries.ptr;
    DftArgs da;
    da.m = a;
    da.rguard = c->d_dft_rguard.ptr;
    da.tguard = c->d_dft_tguard.ptr;
    da.trmax = nullptr; // kTpVar runs the exact epilogue only
    // seed: the Fourier search over one tile per group, one chunk entry per wave (choff = group)
    tp_seed_work<<<(ng + 255) / 256, 256, 0, c->stream>>>(c->d_tp_groups.ptr, ng, c->d_tp_blk_sr.ptr,
                                                          c->d_tp_tile_sd.ptr, c->d_m8_work.ptr);
    FRAC_HIP(c, c->d_m_entries.ensure((size_t)ng * W8 * 64));
    da.m.entries = c->d_m_entries.ptr;
    da.choff = c->d_tp_iota.ptr;
    search_dft<false, kTpVar, W8, 4, true><<<ng, 64 * W8, 0, c->stream>>>(da);
    tp_seed_reduce<<<(nbk * 32 + 255) / 256, 256, 0, c->stream>>>(c->d_tp_blk_group.ptr, c->d_m_entries.ptr,
                                                                   c->d_m_slot_range.ptr, c->d_m_rconst.ptr, nbk,
                                                                   c->d_tp_blk_u.ptr);
    TpWindowArgs w;
    w.groups = c->d_tp_groups.ptr;
    w.ngroups = ng;
    w.blk_sr = c->d_tp_blk_sr.ptr;
    w.blk_u = c->d_tp_blk_u.ptr;
    w.tile_sd = c->d_tp_tile_sd.ptr;
    w.hitH = c->hitH;
    w.work = c->d_m8_work.ptr;
    w.nchunks = c->d_tp_nch.ptr;
    w.pairs = c->d_tp_pairs.ptr;
    FRAC_HIP(c, hipMemsetAsync(c->d_tp_nch.ptr + ng, 0, sizeof(uint32_t), c->stream));
    tp_windows<<<(ng + 255) / 256, 256, 0, c->stream>>>(w);
    size_t tb = c->tp_tmp_bytes;
    FRAC_HIP(c, hipcub::DeviceScan::ExclusiveSum(c->d_tp_tmp.ptr, tb, c->d_tp_nch.ptr, c->d_tp_choff.ptr, (int)(ng + 1),
                                                 c->stream));
    FRAC_HIP(c, hipMemsetAsync(c->d_tp_blkcnt.ptr + nbk, 0, sizeof(uint32_t), c->stream));
    tp_block_counts<<<(nbk + 255) / 256, 256, 0, c->stream>>>(c->d_tp_blk_group.ptr, c->d_tp_nch.ptr, nbk,
                                                              c->d_tp_blkcnt.ptr);
    tb = c->tp_tmp_bytes;
    FRAC_HIP(c, hipcub::DeviceScan::ExclusiveSum(c->d_tp_tmp.ptr, tb, c->d_tp_blkcnt.ptr, c->d_m8_blk_ptr.ptr,
                                                 (int)(nbk + 1), c->stream));
    // sizes of the entry arrays (total chunks, block → entry links) and the searched pairs: one copy
    tp_totals<<<1, 256, 0, c->stream>>>(c->d_tp_choff.ptr, ng, c->d_m8_blk_ptr.ptr, nbk, c->d_tp_pairs.ptr,
                                        c->d_tp_tot.ptr);
    uint32_t tot[4] = {0, 0, 0, 0};
    FRAC_HIP(c, hipMemcpyAsync(tot, c->d_tp_tot.ptr, sizeof(tot), hipMemcpyDeviceToHost, c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    FRAC_HIP(c, c->d_m_entries.ensure(std::max<size_t>((size_t)tot[0] * kDftBlocksPerWG * 64, 1)));
    FRAC_HIP(c, c->d_m8_blk_ent.ensure(std::max<size_t>(tot[1], 1)));
    tp_fill_entries<<<(nbk + 255) / 256, 256, 0, c->stream>>>(c->d_tp_blk_group.ptr, c->d_tp_choff.ptr,
                                                              c->d_m8_blk_ptr.ptr, nbk, c->d_m8_blk_ent.ptr);
    // issued matrix work (8 MFMA 32×32×16 per block × tile) and evaluated (slot, domain row) pairs
    const uint64_t pairs = (uint64_t)tot[2] | ((uint64_t)tot[3] << 32);
    c->flops_ran = pairs * (kDftTpForm == 6 ? 6ull : 8ull) * 32768ull;
    c->evaluated_ran = pairs * 32ull * 32ull;
    da.m.entries = c->d_m_entries.ptr;
    da.choff = c->d_tp_choff.ptr;
    if (c->hitH > 0)
        search_dft<true, kTpVar, W8, 4, true><<<ng, 64 * W8, 0, c->stream>>>(da);
    else
        search_dft<false, kTpVar, W8, 4, true><<<ng, 64 * W8, 0, c->stream>>>(da);
    if (timing)
        FRAC_TRY(mark_event(c, 2));
    MfmaResolveArgs v;
    v.tgt = dtgt;
    v.tstride = tstride;
    v.ranges = c->d_ranges.ptr;
    v.range_slot = c->d_m_range_slot.ptr;
    v.blk_ptr = c->d_m8_blk_ptr.ptr;
    v.blk_ent = c->d_m8_blk_ent.ptr;
    v.entries = c->d_m_entries.ptr;
    v.rconst = c->d_m_rconst.ptr;
    v.tile_pos = c->d_m_tile_pos.ptr;
    v.ntiles = nt;
    v.pool = c->d_pool.ptr;
    v.negsd2 = c->d_negsd2.ptr;
    v.nr = nr;
    v.T = 4;
    v.hitH = c->hitH;
    v.best_key = c->d_best_key.ptr;
    v.slot_range = c->d_m_slot_range.ptr;
    v.nslots = c->nblocks * 32u;
    v.tpool = c->d_dft_tpool.ptr;
    v.rorb = c->d_dft_rorb.ptr;
    FRAC_HIP(c, c->d_rstat.ensure(std::max<size_t>(nr, 1)));
    v.rstat = c->d_rstat.ptr;
    v.fused_fit = 1;
    v.fit = fit_args(c, dtgt, tstride, nr);
    v.fit.tuples = c->qplan ? nullptr : c->tuple_sink;
    c->fit_fused = true;
    // resolve_dft<true> (SORTED) keeps every tie of the ΣD4-ordered chunks but does not merge T = 8's
    // flipped copies (that is the !SORTED path): the tiled form exists for T = 4 only (prepare)
    v.flip_slots = 0;
    if (c->dft_copies != 1 || c->p.transforms != 4)
        return c->fail(FRAC_E_STATE, "SEA tiled form: T = 4 only (resolve_dft<true> has no flipped copies)");
    resolve_dft<true><<<std::max(1u, (v.nslots + 3) / 4), 256, 0, c->stream>>>(v);
    return FRAC_OK;
}

// SEA engine (fracenc_sea.hip): domain keys → radix sort (bucket, ΣD4) → sorted entries;
// range keys → radix sort by ΣR; then one wave per range writes best_key.
template <int N>
int launch_sea(frac_ctx* c, const uint8_t* dtgt, uint32_t tstride, bool timing)
{
    if constexpr (N == 8) {
        if (c->tp)
            return launch_tp(c, dtgt, tstride, timing);
    }
    const uint32_t nr = (uint32_t)nranges(c), P = c->npos * (c->virt ? c->p.transforms : 1u);
    if (P) {
        sea_domain_keys<N><<<(P + 255) / 256, 256, 0, c->stream>>>(c->d_pool.ptr, P, c->d_sea_bend.ptr,
                                                                   (uint32_t)c->bucket_end.size(), c->d_sea_dkey.ptr,
                                                                   c->d_sea_dpos.ptr);
        size_t tb = c->sea_tmp_bytes;
        FRAC_HIP(c, sort_pairs_u32(c->d_sea_tmp.ptr, tb, c->d_sea_dkey.ptr, c->d_sea_dkey2.ptr, c->d_sea_dpos.ptr,
                                   c->d_sea_dpos2.ptr, P, 20, c->stream));
        const uint32_t pieces = (N * N / 2 + 3) / 4;
        sea_domain_entries<N><<<(P * pieces + 255) / 256, 256, 0, c->stream>>>(
            c->d_sea_dkey2.ptr, c->d_sea_dpos2.ptr, c->d_negsd2.ptr, c->d_pool.ptr, P, c->d_sea_ent.ptr,
            c->d_sea_spool.ptr, c->d_sea_snegsd2.ptr);
    }
    if (nr) {
        sea_range_keys<N><<<(nr + 255) / 256, 256, 0, c->stream>>>(dtgt, tstride, c->d_ranges.ptr, nr,
                                                                    c->d_sea_rkey.ptr, c->d_sea_rord.ptr);
        size_t tb = c->sea_tmp_bytes;
        FRAC_HIP(c, sort_pairs_u32(c->d_sea_tmp.ptr, tb, c->d_sea_rkey.ptr, c->d_sea_rkey2.ptr, c->d_sea_rord.ptr,
                                   c->d_sea_rord2.ptr, nr, 17, c->stream));
    }
    if (timing)
        FRAC_TRY(mark_event(c, 1));
    FRAC_HIP(c, hipMemsetAsync(c->d_sea_count.ptr, 0, sizeof(unsigned long long), c->stream));
    if (nr) {
        SeaArgs a;
        a.tgt = dtgt;
        a.tstride = tstride;
        a.ranges = c->d_ranges.ptr;
        a.rbucket = c->d_rbucket.ptr;
        a.rorder = c->d_sea_rord2.ptr;
        a.ent = c->d_sea_ent.ptr;
        a.spool = c->d_sea_spool.ptr;
        a.snegsd2 = c->d_sea_snegsd2.ptr;
        a.nr = nr;
        a.hitH = c->hitH;
        a.best_key = c->d_best_key.ptr;
        a.evaluated = c->d_sea_count.ptr;
        if (c->Teff == 1) // the sampled form: one pool row per (domain, transform)
            sea_search<N, 1><<<(nr + 3) / 4, 256, 0, c->stream>>>(a);
        else if (c->p.transforms == 8)
            sea_search<N, 8><<<(nr + 3) / 4, 256, 0, c->stream>>>(a);
        else
            sea_search<N, 4><<<(nr + 3) / 4, 256, 0, c->stream>>>(a);
    }
    c->form_ran = FRAC_FORM_SEA;
    c->flops_ran = 0;
    return FRAC_OK;
}

// the sampled form's view of the context (fracenc_gen.hip)
GenArgs gen_args(frac_ctx* c, const uint8_t* dtgt, uint32_t tstride)
{
    GenArgs g;
    g.src = c->d_src.ptr;
    g.sstride = c->d_sstride;
    g.tgt = dtgt;
    g.tstride = tstride;
    g.doms = c->d_doms.ptr;
    g.ranges = c->d_ranges.ptr;
    g.porig = c->d_porig.ptr;
    g.nw = c->nw;
    g.nh = c->nh;
    g.Sw = c->Sw;
    g.Sh = c->Sh;
    g.T = c->p.transforms;
    g.K2 = c->K2;
    g.pool = c->d_pool.ptr;
    g.negsd2 = c->d_negsd2.ptr;
    g.nrows = c->npos * c->p.transforms;
    return g;
}

// the sampled form's fit (every range) and fp32 fallback (the flagged ones)
int launch_gen_finish(frac_ctx* c, const GenArgs& g)
{
    const uint32_t nr = (uint32_t)nranges(c);
    if (!nr)
        return FRAC_OK;
    if (!c->all_fallback) {
        GenFitArgs f;
        f.g = g;
        f.best_key = c->d_best_key.ptr;
        f.nr = nr;
        f.hitH = c->hitH;
        f.smax = c->p.s_max;
        f.all_fallback = 0;
        f.out = c->d_out.ptr;
        f.aux = c->d_aux.ptr;
        f.fb_count = c->d_fb_count.ptr;
        f.fb_list = c->d_fb_list.ptr;
        gen_fit<<<(nr + 255) / 256, 256, 0, c->stream>>>(f);
    }
    GenFallbackArgs b;
    b.g = g;
    b.rbucket = c->d_rbucket.ptr;
    b.fb_count = c->d_fb_count.ptr;
    b.fb_list = c->d_fb_list.ptr;
    b.thr = c->p.rms_threshold;
    b.smax = c->p.s_max;
    b.out = c->d_out.ptr;
    b.aux = c->d_aux.ptr;
    gen_fallback<<<512, 256, 0, c->stream>>>(b);
    return FRAC_OK;
}

// range sizes without a templated engine (n ∉ {2, 4, 8, 16}): the sampled form's pool, gen_search,
// gen_fit and gen_fallback
int launch_generic(frac_ctx* c)
{
    const uint32_t nr = (uint32_t)nranges(c);
    const bool timing = (c->p.flags & FRAC_FLAG_TIMING) != 0;
    const uint8_t* dtgt = c->same_plane ? c->d_src.ptr : c->d_tgt.ptr;
    const uint32_t tstride = c->same_plane ? c->d_sstride : c->d_tstride;
    if (timing && c->hist.empty()) {
        c->hist.assign(4 * kHistRuns, nullptr);
        for (size_t i = 0; i < c->hist.size(); ++i)
            FRAC_HIP(c, create_timing_event(&c->hist[i], i));
    }
    if (timing)
        FRAC_TRY(mark_event(c, 0));
    c->fit_fused = false; // gen_fit writes the records; frac_run packs the sink's tuples from them
    c->fb_pending = false;
    if (nr)
        FRAC_HIP(c, hipMemsetAsync(c->d_best_key.ptr, 0xff, nr * sizeof(unsigned long long), c->stream));
    FRAC_HIP(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->d_fb_count.ptr), (int)(c->all_fallback ? nr : 0u),
                                  1, c->stream));
    const GenArgs g = gen_args(c, dtgt, tstride);
    if (g.nrows)
        gen_pool_build<<<(g.nrows + 255) / 256, 256, 0, c->stream>>>(g);
    if (timing)
        FRAC_TRY(mark_event(c, 1));
    if (nr && !c->all_fallback) {
        GenSearchArgs a;
        a.g = g;
        a.rbucket = c->d_rbucket.ptr;
        a.nr = nr;
        a.hitH = c->hitH;
        a.best_key = c->d_best_key.ptr;
        gen_search<<<(nr + 3) / 4, 256, 0, c->stream>>>(a);
    }
    if (timing)
        FRAC_TRY(mark_event(c, 2));
    FRAC_TRY(launch_gen_finish(c, g));
    if (timing) {
        FRAC_TRY(mark_event(c, 3));
        ++c->hist_runs;
    }
    FRAC_HIP(c, hipGetLastError());
    c->engine_ran = FRAC_ENGINE_VALU;
    c->form_ran = FRAC_FORM_SAMPLED;
    c->flops_ran = 0;
    c->evaluated_ran = c->all_fallback ? 0 : c->eligible_pairs;
    return FRAC_OK;
}

template <int N>
int launch_all(frac_ctx* c)
{
    const uint32_t nr = (uint32_t)nranges(c), P = c->npos * (c->virt ? c->p.transforms : 1u);
    const bool timing = (c->p.flags & FRAC_FLAG_TIMING) != 0;
    const uint8_t* dsrc = c->d_src.ptr;
    const uint8_t* dtgt = c->same_plane ? c->d_src.ptr : c->d_tgt.ptr;
    const uint32_t tstride = c->same_plane ? c->d_sstride : c->d_tstride;
    HostTrace tr("launch");
    if (timing && c->hist.empty()) {
        c->hist.assign(4 * kHistRuns, nullptr);
        for (size_t i = 0; i < c->hist.size(); ++i)
            FRAC_HIP(c, create_timing_event(&c->hist[i], i));
    }
    if (timing)
        FRAC_TRY(mark_event(c, 0));
    c->fit_rstat = false;
    c->fit_fused = false;
    const bool use_mfma = c->engine == FRAC_ENGINE_MFMA && !c->all_fallback;
    // the Fourier path resets best_key and fb_count in its preparation kernel (dft_prep)
    const bool dft_inits = N == 8 && use_mfma && nr && dft_route(c);
    if (!dft_inits && !c->qplan) { // (a planned level's qt_fill_maps did both)
        if (nr)
            FRAC_HIP(c, hipMemsetAsync(c->d_best_key.ptr, 0xff, nr * sizeof(unsigned long long), c->stream));
        const uint32_t fbc = c->all_fallback ? nr : 0u;
        // a device-side fill, not an H2D copy from pageable host memory (which serialises the host
        // with the stream)
        FRAC_HIP(c, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(c->d_fb_count.ptr), (int)fbc, 1, c->stream));
    }
    // the Fourier path and the SEA engine's tiled form build the pool in their fused domain pass
    // (dft_domain_build)
    // (and the direct form at n = 4 / 16 in mfma_prep's domain half)
    const bool fused_pool = !c->virt &&
                            ((N == 8 && ((use_mfma && (c->p.transforms == 4 || c->dft_copies == 2) && mfma_dft_enabled(c)) ||
                                         (c->engine == FRAC_ENGINE_SEA && !c->all_fallback && c->tp))) ||
                             ((N == 4 || N == 16) && use_mfma));
    const GenArgs g = gen_args(c, dtgt, tstride);
    if (P && c->virt) // the sampled form: one row per (domain, transform), fracenc_gen.hip
        gen_pool_build<<<(P + 255) / 256, 256, 0, c->stream>>>(g);
    else if (P && !fused_pool) { // pool_lanes<N>() lanes per pool position
        const unsigned nblk = (unsigned)(((uint64_t)P * pool_lanes<N>() + 255) / 256);
        pool_build<N><<<nblk, 256, 0, c->stream>>>(dsrc, c->d_sstride, c->d_doms.ptr, c->d_porig.ptr, P, c->d_pool.ptr,
                                                   c->d_negsd2.ptr);
    }
    const bool use_sea = c->engine == FRAC_ENGINE_SEA && !c->all_fallback;
    tr.mark("memsets + pool");
    if (use_mfma)
        FRAC_TRY(launch_mfma<N>(c, dtgt, tstride, dft_inits));
    if constexpr (N <= 8) {
        if (use_sea)
            FRAC_TRY(launch_sea<N>(c, dtgt, tstride, timing));
    }
    tr.mark("engine launch");
    const bool use_valu = !use_mfma && !use_sea;
    if (timing && use_valu)
        FRAC_TRY(mark_event(c, 1));
    if (use_valu && !c->all_fallback && !c->work.empty()) {
        SearchArgs a;
        a.tgt = dtgt;
        a.tstride = tstride;
        a.ranges = c->d_ranges.ptr;
        a.slot_range = c->d_slot_range.ptr;
        a.pool = c->d_pool.ptr;
        a.negsd2 = c->d_negsd2.ptr;
        a.work = c->d_work.ptr;
        a.nwork = (uint32_t)c->work.size();
        a.hitH = (int32_t)std::max<int64_t>(c->hitH, 0);
        a.best_key = c->d_best_key.ptr;
        const dim3 grid((a.nwork + 3) / 4), block(256);
        const bool hits = c->hitH > 0; // H = 0: the first maximum of w is the first hit
        if (N == 16 || c->G == 1) { // one copy: n = 16, or the sampled form's identity transform
            if (hits)
                search_valu<N, 1, true><<<grid, block, 0, c->stream>>>(a);
            else
                search_valu<N, 1, false><<<grid, block, 0, c->stream>>>(a);
        } else if constexpr (N <= 4) {
            if (c->G == 8) {
                if (hits)
                    search_valu<N, 8, true><<<grid, block, 0, c->stream>>>(a);
                else
                    search_valu<N, 8, false><<<grid, block, 0, c->stream>>>(a);
            } else {
                if (hits)
                    search_valu<N, 4, true><<<grid, block, 0, c->stream>>>(a);
                else
                    search_valu<N, 4, false><<<grid, block, 0, c->stream>>>(a);
            }
        } else if constexpr (N < 16) { // n = 16 never takes a 4-copy group (4 × 128 words of copies would spill)
            if (hits)
                search_valu<N, 4, true><<<grid, block, 0, c->stream>>>(a);
            else
                search_valu<N, 4, false><<<grid, block, 0, c->stream>>>(a);
        }
    }
    if (timing && !use_mfma)
        FRAC_TRY(mark_event(c, 2));
    if (c->virt) {
        FRAC_TRY(launch_gen_finish(c, g));
    } else if (!c->all_fallback && nr && !c->fit_fused) {
        FitArgs f = fit_args(c, dtgt, tstride, nr);
        if (c->fit_rstat)
            fit_rstat<N><<<(nr + 255) / 256, 256, 0, c->stream>>>(f, c->d_rstat.ptr);
        else
            fit_winner<N><<<std::max(1u, (nr + 4 * (64 / fit_lanes<N>()) - 1) / (4 * (64 / fit_lanes<N>()))), 256, 0,
                            c->stream>>>(f);
    }
    // the fp32 fallback: the fused resolvers (n ≥ 8; below no range leaves the exact regime) list their
    // fp32-regime ranges and fallback_grid settles them before the records are read (settle_fallback); every
    // other path runs it here
    c->fb_pending = false;
    if (nr && !c->virt) {
        FRAC_TRY(ensure_fb_scratch(c));
        const FallbackArgs b = fallback_args(c, dtgt, tstride);
        if (c->fit_fused && !c->all_fallback) {
            if constexpr (N >= 8) {
                c->fb_pending = true;
                c->fb_n = N;
                c->fb_args = b;
            }
        } else {
            launch_fallback_grid<N>(c, b);
        }
    }
    if (timing) {
        FRAC_TRY(mark_event(c, 3));
        ++c->hist_runs;
    }
    FRAC_HIP(c, hipGetLastError());
    tr.mark("fit + fallback");
    c->engine_ran = use_mfma ? FRAC_ENGINE_MFMA : use_sea ? FRAC_ENGINE_SEA : FRAC_ENGINE_VALU;
    if (!(use_sea && c->tp)) // the tiled form counted its evaluated pairs in launch_tp
        c->evaluated_ran = c->all_fallback ? 0 : c->eligible_pairs; // SEA: read back at fetch
    if (use_valu) {
        c->form_ran = FRAC_FORM_DOT2;
        c->flops_ran = 0;
    }
    return FRAC_OK;
}

// every level's domain grid (geometry only) stays on the host and the device across frames: the
// level swaps them in (no copy, no upload, no re-validation) and back out afterwards
// the caller's domain-list state comes back afterwards; the range list is consumed (cleared, unset)
struct LevelGrid {
    frac_ctx* c;
    bool doms_set_before;
    int lv = -1;
    void in(int level)
    {
        lv = level;
        std::swap(c->doms, c->qt_doms[lv]);
        std::swap(c->d_doms, c->qt_ddoms[lv]);
        c->doms_set = true;
        c->doms_uploaded = c->qt_dvalid[lv];
        c->doms_trusted = true;
        c->dirty = true;
    }
    void out()
    {
        if (lv < 0)
            return;
        c->qt_dvalid[lv] = c->doms_uploaded;
        std::swap(c->doms, c->qt_doms[lv]);
        std::swap(c->d_doms, c->qt_ddoms[lv]);
        c->doms_uploaded = false;
        c->doms_trusted = false;
        c->dirty = true;
        lv = -1;
    }
    ~LevelGrid()
    {
        out();
        c->ranges_dev = false;
        c->doms_set = doms_set_before;
        c->ranges_set = false;
    }
};

// Whether a quadtree frame runs device-planned (qt_encode_dev): the MFMA engine at every level (AUTO
// or MFMA requested; the VALU and SEA engines keep the host-planned levels below), and no level in
// the all-fallback regime (a threshold that can be met in the inexact regime).
bool qt_device_planned(const frac_ctx* c, const frac_quadtree_params* qp)
{
    if (c->p.engine != FRAC_ENGINE_AUTO && c->p.engine != FRAC_ENGINE_MFMA)
        return false;
    // the planner hard-codes the shipped layouts (8-wave Fourier work items, the default direct variants):
    // a tuning build with an A/B knob set runs the host-planned levels, which honour it
    if (kTuningBuild)
        for (const char* k : kAbKnobs) {
            const char* v = getenv(k);
            if (v && *v)
                return false;
        }
    for (uint32_t n = qp->max_size; n >= qp->min_size; n /= 2)
        if (compute_hit_limit(c->p.rms_threshold, 4 * n * n) >= kExactLimit)
            return false;
    return true;
}

// A quadtree frame with every level laid out on the device (fracenc_bucket.hip qt_plan): per level the
// domain and range bucket keys, sorts and bounds, the planner (layout, work lists, CSR map, counts
// into the level's DevPlan), qt_fill_maps, the level's search (launch_all in plan mode: worst-case
// grids whose surplus workgroups leave at once) and the level transition (qt_flags, scan, qt_scatter,
// which writes the next level's count into the next DevPlan).  Nothing comes back to the host until
// the frame is done: one synchronisation for the leaf count and the counters, one for the leaves —
// where the host-planned path synchronised twice per level (bucket counts, split count).  Records,
// leaves and counters are those of the host-planned path.
// the frame's counters (qt_level_stats, qt_plan): {rejected, hit, fallback, empty, -, total, eligible,
// flops, overflow} in kQtShards copies, summed by the host
constexpr uint32_t kQtShards = 32, kQtCounters = 9;

int qt_encode_dev(frac_ctx* c, const frac_quadtree_params* qp, LevelGrid& level, frac_encode_item* out, size_t cap,
                  size_t* n_out, frac_stats* stats, frac_qt_leaf* out32 = nullptr)
{
    const uint32_t W = c->src.w, H = c->src.h, T = c->p.transforms;
    const int nb = c->p.use_classifier ? 7 : 1;
    const bool timing = (c->p.flags & FRAC_FLAG_TIMING) != 0;
    const uint8_t* tplane = c->same_plane ? c->d_src.ptr : c->d_tgt.ptr;
    const uint32_t tstride = c->same_plane ? c->d_sstride : c->d_tstride;
    HostTrace tr("quadtree (device-planned)");
    const size_t max_leaves = (size_t)(W / qp->min_size) * (H / qp->min_size);
    constexpr uint32_t kFirst = 2 * (kMaxBuckets + 1); // bucket bounds per level: domains, ranges
    if (out32)
        FRAC_HIP(c, c->d_qt_leaves32.ensure(std::max<size_t>(max_leaves, 1)));
    else
        FRAC_HIP(c, c->d_qt_leaves.ensure(std::max<size_t>(max_leaves, 1)));
    FRAC_HIP(c, c->d_ranges.ensure(std::max<size_t>(max_leaves, 1)));
    FRAC_HIP(c, c->d_qt_next.ensure(std::max<size_t>(max_leaves, 1)));
    FRAC_HIP(c, c->d_qt_plan.ensure(6));
    FRAC_HIP(c, c->d_qt_first.ensure(5 * kFirst));
    FRAC_HIP(c, c->d_qt_stats.ensure(kQtShards * kQtCounters));
    FRAC_HIP(c, c->d_bk_first.ensure(2 * (kMaxBuckets + 1) + 1));
    // the classifier keys of every level from the frame's block sums, summed once here (domains 2n ≤ 32 rows)
    BlockSums bs_src, bs_tgt;
    const bool use_bs = nb > 1 && qp->max_size <= 16;
    if (use_bs)
        FRAC_TRY(plane_block_sums(c, bs_src, bs_tgt));
    // the first level's ranges: createUniformGrid(W, H, max, max), generated on the device
    const uint32_t m0 = qp->max_size;
    const uint32_t nr0 = W >= m0 && H >= m0 ? ((W - m0) / m0 + 1) * ((H - m0) / m0 + 1) : 0u;
    // (the same launch zeroes the frame's counters)
    constexpr uint32_t kQtZero = kQtShards * kQtCounters;
    qt_uniform_grid<<<(std::max(nr0, kQtZero) + 255) / 256, 256, 0, c->stream>>>(
        nr0 ? (W - qp->max_size) / qp->max_size + 1 : 1u, nr0, qp->max_size, qp->max_size, c->d_ranges.ptr,
        c->d_qt_stats.ptr, kQtZero);
    // the leaves go straight into the caller's buffer when it is pinned host memory the device can write
    // (the emit kernels write them over PCIe while the later levels run); else into d_qt_leaves and one
    // copy at the end
    frac_encode_item* leaves = c->d_qt_leaves.ptr;
    frac_qt_leaf* leaves32 = out32 ? c->d_qt_leaves32.ptr : nullptr;
    uint32_t leaf_cap = (uint32_t)std::min<size_t>(max_leaves, 0xffffffffu);
    bool direct = false;
    void* const host_out = out32 ? static_cast<void*>(out32) : static_cast<void*>(out);
    if (host_out && cap) {
        hipPointerAttribute_t at{};
        void* dp = nullptr;
        if (hipPointerGetAttributes(&at, host_out) == hipSuccess && at.type == hipMemoryTypeHost &&
            hipHostGetDevicePointer(&dp, host_out, 0) == hipSuccess && dp) {
            if (out32)
                leaves32 = reinterpret_cast<frac_qt_leaf*>(dp);
            else
                leaves = reinterpret_cast<frac_encode_item*>(dp);
            leaf_cap = (uint32_t)std::min<size_t>(cap, 0xffffffffu);
            direct = true;
        }
        (void)hipGetLastError(); // pageable memory is not an error
    }
    if (!c->h_qt_sum)
        FRAC_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_qt_sum), sizeof(QtFrameSum)));
    uint32_t nr_bound = nr0; // the level's worst-case range count
    int lvi = 0;             // level index (plans 0..4; plan lvi + 1 receives the next count)
    std::vector<uint64_t> runs; // the levels' timing-history runs
    for (uint32_t n = qp->max_size; n >= qp->min_size && nr_bound; n /= 2, ++lvi) {
        const int lv = __builtin_ctz(n);
        if (c->qt_doms[lv].empty()) {
            c->qt_doms[lv].resize(frac_uniform_grid(W, H, 2 * n, n, nullptr, 0));
            if (!c->qt_doms[lv].empty())
                frac_uniform_grid(W, H, 2 * n, n, c->qt_doms[lv].data(), c->qt_doms[lv].size());
        }
        level.in(lv);
        const uint32_t nd = (uint32_t)c->doms.size(), nr_max = nr_bound;
        FRAC_HIP(c, c->d_doms.ensure(std::max<uint32_t>(nd, 1)));
        if (!c->doms_uploaded && nd) {
            FRAC_HIP(c, hipMemcpyAsync(c->d_doms.ptr, c->doms.data(), nd * sizeof(frac_grid_item),
                                       hipMemcpyHostToDevice, c->stream));
            c->doms_uploaded = true;
        }
        // the level's geometry (prepare()'s fields for a ratio-2 square level on the MFMA engine)
        c->n = (int)n;
        c->S = c->Sw = c->Sh = 2 * n;
        c->nw = c->nh = n;
        c->virt = c->generic = false;
        c->Teff = T;
        c->K2 = n * n / 2;
        c->G = n == 16 ? 1u : (n <= 4 ? T : 4u);
        c->NG = T / c->G;
        c->npos = nd;
        c->engine = FRAC_ENGINE_MFMA;
        c->tp = false;
        c->hitH = compute_hit_limit(c->p.rms_threshold, 4 * n * n);
        c->all_fallback = false;
        const bool fourier = n == 8 && mfma_dft_enabled(c);
        c->dft_copies = fourier && T == 8 ? 2u : 1u;
        const uint32_t cp = c->dft_copies, KS = (n * n + 15) / 16;
        const uint32_t bpw = n == 16 ? mfma16_bpw(T) : fourier ? kDftBlocksPerWG : 4u;
        const uint32_t target = n == 16 ? kMfma16TargetWgs : fourier ? 8192u / kDftBlocksPerWG * 4u : 8192u;
        const uint32_t nblocks_cap = (nr_max + 31) / 32 + (uint32_t)nb;
        const uint32_t ntiles_cap = (nd + 31) / 32 + (uint32_t)nb;
        const uint32_t groups_cap = (nblocks_cap * cp + bpw - 1) / bpw + (uint32_t)nb * cp;
        const uint32_t nwork_cap = target + groups_cap, nent_cap = bpw * nwork_cap;
        // buffers at the level's bounds (kept across frames: ensure() reallocates only to grow)
        const size_t mx = std::max<size_t>(std::max<size_t>(nd, nr_max), 1);
        FRAC_HIP(c, c->d_porig.ensure(std::max<uint32_t>(nd, 1)));
        FRAC_HIP(c, c->d_pool.ensure((size_t)std::max<uint32_t>(nd, 1) * c->K2));
        FRAC_HIP(c, c->d_negsd2.ensure(std::max<uint32_t>(nd, 1)));
        for (auto* b : {&c->d_rord, &c->d_rkey, &c->d_fb_list, &c->d_m_range_slot, &c->d_qt_flags, &c->d_qt_offs})
            FRAC_HIP(c, b->ensure(std::max<uint32_t>(nr_max, 1)));
        FRAC_HIP(c, c->d_rbucket.ensure(std::max<uint32_t>(nr_max, 1)));
        FRAC_HIP(c, c->d_best_key.ensure(std::max<uint32_t>(nr_max, 1)));
        FRAC_HIP(c, c->d_out.ensure(std::max<uint32_t>(nr_max, 1)));
        FRAC_HIP(c, c->d_aux.ensure(std::max<uint32_t>(nr_max, 1)));
        FRAC_HIP(c, c->d_fb_count.ensure(1));
        FRAC_HIP(c, c->d_bk_keys.ensure(mx));
        FRAC_HIP(c, c->d_m_slot_range.ensure((size_t)nblocks_cap * 32 * cp));
        FRAC_HIP(c, c->d_m_rconst.ensure((size_t)nblocks_cap * 32 * cp));
        FRAC_HIP(c, c->d_m_tile_pos.ensure((size_t)ntiles_cap * 32));
        FRAC_HIP(c, c->d_m_dconst.ensure((size_t)ntiles_cap * kDftCS * 4 + 256));
        FRAC_HIP(c, c->d_m_dtiles.ensure((size_t)ntiles_cap * std::max(KS, 5u) * 64));
        FRAC_HIP(c, c->d_m_rfrags.ensure((size_t)nblocks_cap * std::max(T * KS, 6u * cp) * 64));
        DBuf<uint4>& dwork = fourier ? c->d_m8_work : c->d_m_work;
        DBuf<uint32_t>& dptr = fourier ? c->d_m8_blk_ptr : c->d_m_blk_ptr;
        DBuf<uint32_t>& dent = fourier ? c->d_m8_blk_ent : c->d_m_blk_ent;
        FRAC_HIP(c, dwork.ensure(nwork_cap));
        FRAC_HIP(c, dptr.ensure((size_t)nblocks_cap * cp + 1));
        FRAC_HIP(c, dent.ensure(std::max<uint32_t>(nent_cap, 1)));
        FRAC_HIP(c, c->d_m_entries.ensure((size_t)nwork_cap * (fourier ? kDftBlocksPerWG : 4u * T) * 64));
        FRAC_HIP(c, c->d_bk_cnt.ensure(((size_t)(nd + kBkTile - 1) / kBkTile + (nr_max + kBkTile - 1) / kBkTile + 2) *
                                       kMaxBuckets));
        tr.mark("level buffers");
        DevPlan* plan = c->d_qt_plan.ptr + lvi;
        const uint32_t* dn = lvi ? &plan->nr : nullptr; // the first level's count is the host's
        uint32_t* first = c->d_qt_first.ptr + (size_t)lv * kFirst;
        if (nb > 1) {
            // domains: keys + stable bucket sort (the pool order porig) + bounds; ranges: the same over the
            // worst case, counting only the level's *dn (the grids' categories are −1, computed here:
            // no invalid category can occur, so no error word)
            const KeySeg kd{c->d_doms.ptr, nd, c->d_src.ptr, c->d_sstride, c->d_bk_keys.ptr, nullptr, nullptr, nullptr};
            const KeySeg kr{c->d_ranges.ptr, nr_max, tplane, tstride, c->d_rkey.ptr, nullptr, nullptr, dn};
            if (use_bs) // the frame's block sums, summed once before the first level
                launch_bucket_keys_bs(kd, bs_src, 2 * n, 2 * n, kr, bs_tgt, n, n, c->stream);
            else
                launch_bucket_keys_pair(kd, 2 * n, kr, n, c->stream);
            // both sorts in one set of launches (the range counts after the domain counts in the scratch)
            const BkSeg sd = bk_seg_of(c->d_bk_keys.ptr, nd, nullptr, c->d_bk_cnt.ptr, first, c->d_porig.ptr);
            const BkSeg sr = bk_seg_of(c->d_rkey.ptr, nr_max, dn, c->d_bk_cnt.ptr + (size_t)sd.tiles * kMaxBuckets,
                                       first + kMaxBuckets + 1, c->d_rord.ptr);
            launch_bucket_sorts(sd, sr, c->stream);
        } else {
            if (nd)
                fill_iota<<<(nd + 255) / 256, 256, 0, c->stream>>>(c->d_porig.ptr, nd);
            fill_iota<<<(nr_max + 255) / 256, 256, 0, c->stream>>>(c->d_rord.ptr, nr_max);
            FRAC_HIP(c, hipMemsetAsync(c->d_rkey.ptr, 0, nr_max * sizeof(uint32_t), c->stream));
        }
        QtPlanArgs pa;
        pa.plan = plan;
        pa.dfirst = nb > 1 ? first : nullptr;
        pa.rfirst = nb > 1 ? first + kMaxBuckets + 1 : nullptr;
        pa.nb = (uint32_t)nb;
        pa.nd = nd;
        pa.nr_init = lvi ? ~0u : nr0;
        pa.bpw = bpw;
        pa.target = target;
        pa.copies = cp;
        pa.mfma_per_pair = fourier ? 6u : T * KS;
        pa.nwork_cap = nwork_cap;
        pa.nent_cap = nent_cap;
        pa.nblocks_cap = nblocks_cap;
        pa.ntiles_cap = ntiles_cap;
        pa.work = dwork.ptr;
        pa.blk_ptr = dptr.ptr;
        pa.blk_ent = dent.ptr;
        pa.acc = c->d_qt_stats.ptr;
        QtFillArgs& fa = pa.fill;
        fa.rord = c->d_rord.ptr;
        fa.rkey = c->d_rkey.ptr;
        fa.copies = cp;
        fa.nthreads = std::max(std::max(nblocks_cap * 32 * cp, ntiles_cap * 32), nr_max);
        fa.slot_range = c->d_m_slot_range.ptr;
        fa.range_slot = c->d_m_range_slot.ptr;
        fa.tile_pos = c->d_m_tile_pos.ptr;
        fa.rbucket = c->d_rbucket.ptr;
        fa.rconst = fourier ? nullptr : c->d_m_rconst.ptr;
        fa.best_key = c->d_best_key.ptr;
        fa.fb_count = c->d_fb_count.ptr;
        // the layout, work lists, CSR map and per-item maps: one launch
        qt_plan<<<std::max(32u, (fa.nthreads + 255) / 256), 256, 0, c->stream>>>(pa);
        // the level's search, on the bounds: launch_all in plan mode
        c->m_work.clear();
        c->m8_work.clear();
        c->ranges_dev = true;
        c->nr_dev = nr_max;
        c->n_dev = n;
        c->ntiles = ntiles_cap;
        c->nblocks = nblocks_cap;
        c->m8_bpw = kDftBlocksPerWG;
        c->qplan = plan;
        c->qp_nwork_cap = nwork_cap;
        int rc;
        switch (n) {
        case 2: rc = launch_all<2>(c); break;
        case 4: rc = launch_all<4>(c); break;
        case 16: rc = launch_all<16>(c); break;
        default: rc = launch_all<8>(c); break;
        }
        c->qplan = nullptr;
        FRAC_TRY(rc);
        FRAC_TRY(settle_fallback(c)); // the level's records are complete before its transition reads them
        if (timing)
            runs.push_back(c->hist_runs - 1);
        tr.mark("level launch");
        level.out();
        // the level transition: split counts and counters, their prefix and the next count, leaves and quadrants
        QtSplitArgs sa;
        sa.out = c->d_out.ptr;
        sa.ranges = c->d_ranges.ptr;
        sa.plan = plan;
        sa.next = plan + 1;
        sa.nmax = nr_max;
        sa.can_split = n > qp->min_size ? 1 : 0;
        sa.split = qp->split_distance;
        sa.tcount = c->d_qt_flags.ptr;
        // (a second stream copying a level's leaves across PCIe while the next level ran measured slower: the
        // copy kernel's PCIe writes stalled the next level's bucket keys 11 → 71 µs)
        sa.leaves = leaves;
        sa.leaves32 = leaves32;
        sa.dcols = W >= 2 * n ? (W - 2 * n) / n + 1 : 0u;
        sa.leaf_cap = leaf_cap;
        sa.next_ranges = c->d_qt_next.ptr;
        sa.aux = c->d_aux.ptr;
        sa.rkey = c->d_rkey.ptr;
        sa.porig = c->d_porig.ptr;
        sa.nd = nd;
        sa.classifier = c->p.use_classifier ? 1 : 0;
        sa.acc = stats ? c->d_qt_stats.ptr : nullptr;
        sa.shards = kQtShards;
        sa.stride = kQtCounters;
        const uint32_t ntl = std::max<uint32_t>((nr_max + kBkTile - 1) / kBkTile, 1u);
        qt_split_count<<<ntl, kBkThreads, 0, c->stream>>>(sa);
        qt_split_emit<<<ntl, kBkThreads, 0, c->stream>>>(sa);
        std::swap(c->d_ranges, c->d_qt_next);
        // the next level: at most four quadrants per range, at most the full grid of its size (counted in
        // closed form: frac_uniform_grid's count loop took 0.2 ms of host time for the 2×2 grid at 2048²)
        auto grid_count = [&](uint32_t size) -> uint32_t {
            return W >= size && H >= size ? ((W - size) / size + 1) * ((H - size) / size + 1) : 0u;
        };
        nr_bound = n > qp->min_size ? std::min<uint32_t>(4 * nr_max, grid_count(n / 2)) : 0u;
        tr.mark("split (device)");
    }
    c->ranges_dev = false;
    c->ranges.clear();
    c->ranges_set = false;
    c->dirty = true;
    c->ran = false;
    // the frame's one round trip: qt_finish writes the leaf count and the summed counters into pinned
    // memory (the leaves are already in the caller's buffer when it is pinned)
    void* dsum = nullptr;
    FRAC_HIP(c, hipHostGetDevicePointer(&dsum, c->h_qt_sum, 0));
    qt_finish<<<1, 64, 0, c->stream>>>(c->d_qt_plan.ptr + lvi, lvi ? 1 : 0, c->d_qt_stats.ptr, kQtShards, kQtCounters,
                                       reinterpret_cast<QtFrameSum*>(dsum));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    struct {
        unsigned long long acc[kQtCounters];
    } h{};
    for (uint32_t i = 0; i < kQtCounters; ++i)
        h.acc[i] = c->h_qt_sum->acc[i];
    if (h.acc[8])
        return c->fail(FRAC_E_STATE, "quadtree: a level's layout exceeded its planned bounds");
    const uint32_t n_leaves = c->h_qt_sum->leaves;
    *n_out = n_leaves;
    if (out && n_leaves && !direct)
        FRAC_HIP(c, hipMemcpy(out, c->d_qt_leaves.ptr, std::min<size_t>(cap, n_leaves) * sizeof(frac_encode_item),
                              hipMemcpyDeviceToHost));
    if (out32 && n_leaves && !direct)
        FRAC_HIP(c, hipMemcpy(out32, c->d_qt_leaves32.ptr, std::min<size_t>(cap, n_leaves) * sizeof(frac_qt_leaf),
                              hipMemcpyDeviceToHost));
    tr.mark("leaves D2H");
    if (stats) {
        frac_stats total{};
        total.rejected_mappings = h.acc[0];
        total.hit_ranges = (uint32_t)h.acc[1];
        total.fallback_ranges = (uint32_t)h.acc[2];
        total.empty_ranges = (uint32_t)h.acc[3];
        total.total_mappings = h.acc[5];
        total.evaluated_mappings = h.acc[6];
        total.matrix_flops = h.acc[7];
        total.engine = FRAC_ENGINE_MFMA;
        total.search_form = c->form_ran;
        if (timing)
            for (uint64_t r : runs) {
                hipEvent_t* e = &c->hist[(size_t)(r % kHistRuns) * 4];
                float ms = 0.f;
                if (hipEventElapsedTime(&ms, e[0], e[3]) == hipSuccess)
                    total.ms_device += ms;
                if (hipEventElapsedTime(&ms, e[0], e[1]) == hipSuccess)
                    total.ms_prep += ms;
                if (hipEventElapsedTime(&ms, e[1], e[2]) == hipSuccess)
                    total.ms_search += ms;
                if (hipEventElapsedTime(&ms, e[2], e[3]) == hipSuccess)
                    total.ms_finish += ms;
            }
        *stats = total;
    }
    return FRAC_OK;
}
} // namespace

extern "C" {

int frac_abi_version(void) { return FRAC_ABI_VERSION; }

int frac_device_count(void)
{
    int count = 0;
    const hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess) {
        g_last_error = std::string("hipGetDeviceCount: ") + hipGetErrorString(e);
        return FRAC_E_DEVICE;
    }
    return count;
}

// The source id build() compiles in (-DFRAC_SOURCE_ID="…": the hash fractencode_amd.source_id()
// computes over csrc/ and include/fracenc.h), so a result can name the binary that produced it.
#ifndef FRAC_SOURCE_ID
#define FRAC_SOURCE_ID "unknown"
#endif
const char* frac_build_id(void) { return FRAC_SOURCE_ID; }

int frac_build_flags(void) { return kTuningBuild ? FRAC_BUILD_TUNING : 0; }

const char* frac_last_error(const frac_ctx* ctx) { return ctx ? ctx->err.c_str() : g_last_error.c_str(); }

frac_ctx* frac_create(int device, const frac_params* params)
{
    std::string msg;
    if (check_params(params, msg) != FRAC_OK) {
        g_last_error = msg;
        return nullptr;
    }
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) {
        g_last_error = std::string("no HIP device: ") + hipGetErrorString(e);
        return nullptr;
    }
    if (device < 0 || device >= count) {
        g_last_error = "device index out of range";
        return nullptr;
    }
    e = hipSetDevice(device);
    if (e != hipSuccess) {
        g_last_error = std::string("hipSetDevice: ") + hipGetErrorString(e);
        return nullptr;
    }
    auto* c = new frac_ctx();
    c->device = device;
    c->p = *params;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
        g_last_error = "hipStreamCreate failed";
        delete c;
        return nullptr;
    }
    c->stream = c->own_stream;
    for (size_t k = 0; k < 5; ++k)
        if ((k < 4 ? create_timing_event(&c->ev[k], k) : hipEventCreate(&c->ev[k])) != hipSuccess) {
            g_last_error = "hipEventCreate failed";
            frac_destroy(c);
            return nullptr;
        }
    return c;
}

void frac_destroy(frac_ctx* c)
{
    if (!c)
        return;
    (void)hipSetDevice(c->device);
    if (c->stream)
        (void)hipStreamSynchronize(c->stream);
    c->d_src.release();
    c->d_tgt.release();
    if (c->copy_stream)
        (void)hipStreamSynchronize(c->copy_stream);
    c->d_src_next.release();
    c->d_doms.release();
    c->d_ranges.release();
    c->d_porig.release();
    c->d_pool.release();
    c->d_fb_list.release();
    c->d_fb_count.release();
    c->d_negsd2.release();
    c->d_slot_range.release();
    c->d_work.release();
    c->d_rbucket.release();
    c->d_best_key.release();
    c->d_out.release();
    c->d_aux.release();
    c->d_m_slot_range.release();
    c->d_m_tile_pos.release();
    c->d_m_range_slot.release();
    c->d_m_blk_ptr.release();
    c->d_m_blk_ent.release();
    c->d_m_rconst.release();
    c->d_m_dconst.release();
    c->d_m_work.release();
    c->d_m8_work.release();
    c->d_m8_blk_ptr.release();
    c->d_m8_blk_ent.release();
    c->d_m_dtiles.release();
    c->d_m_rfrags.release();
    c->d_sea_dkey.release();
    c->d_sea_dkey2.release();
    c->d_sea_dpos.release();
    c->d_sea_dpos2.release();
    c->d_sea_rkey.release();
    c->d_sea_rkey2.release();
    c->d_sea_rord.release();
    c->d_sea_rord2.release();
    c->d_sea_bend.release();
    c->d_sea_spool.release();
    c->d_sea_count.release();
    c->d_sea_snegsd2.release();
    c->d_tuples.release();
    c->d_tp_groups.release();
    c->d_tp_blk_group.release();
    c->d_tp_tile_sd.release();
    c->d_tp_blk_sr.release();
    c->d_tp_blk_u.release();
    c->d_tp_nch.release();
    c->d_tp_choff.release();
    c->d_tp_blkcnt.release();
    c->d_tp_tot.release();
    c->d_tp_pairs.release();
    c->d_tp_row_of.release();
    c->d_tp_iota.release();
    c->d_tp_rbk.release();
    c->d_tp_tmp.release();
    c->d_frc_mm.release();
    c->d_frc_rec.release();
    c->d_frc_words.release();
    c->d_sea_ent.release();
    c->d_sea_tmp.release();
    c->d_m_entries.release();
    c->d_dec_src.release();
    c->d_color.release();
    c->d_dec_part.release();
    c->d_dec_state.release();
    if (c->h_dec_state)
        (void)hipHostFree(c->h_dec_state);
    c->d_dft_tguard.release();
    c->d_dft_trmax.release();
    c->d_dft_tpool.release();
    c->d_dft_rorb.release();
    c->d_dft_slotbest.release();
    c->d_qt_leaves32.release();
    c->d_fb_key.release();
    c->d_fb_done.release();
    c->d_rstat.release();
    c->d_cls_items.release();
    c->d_cls_list.release();
    c->d_cls_out.release();
    c->d_dft_rguard.release();
    c->d_dec_tgt.release();
    c->d_rord.release();
    for (auto& q : c->qt_ddoms)
        q.release();
    c->d_qt_next.release();
    c->d_qt_leaves.release();
    c->d_qt_flags.release();
    c->d_qt_offs.release();
    c->d_qt_count.release();
    c->d_qt_stats.release();
    c->d_qt_tmp.release();
    c->d_rkey.release();
    c->d_bk_keys.release();
    c->d_bk_cnt.release();
    c->d_bsum_s.release();
    c->d_bsum_t.release();
    c->d_bk_keys2.release();
    c->d_bk_iota.release();
    c->d_bk_first.release();
    c->d_bk_err.release();
    c->d_bk_tmp.release();
    c->d_dec_items.release();
    c->d_dec_sum.release();
    if (c->h_dec_sum)
        (void)hipHostFree(c->h_dec_sum);
    if (c->h_qt_sum)
        (void)hipHostFree(c->h_qt_sum);
    for (auto& ev : c->ev)
        if (ev)
            (void)hipEventDestroy(ev);
    if (c->handoff)
        (void)hipEventDestroy(c->handoff);
    for (auto& ev : c->hist)
        if (ev)
            (void)hipEventDestroy(ev);
    if (c->own_stream)
        (void)hipStreamDestroy(c->own_stream);
    if (c->copy_stream)
        (void)hipStreamDestroy(c->copy_stream);
    if (c->up_done)
        (void)hipEventDestroy(c->up_done);
    if (c->next_free)
        (void)hipEventDestroy(c->next_free);
    delete c;
}

int frac_set_params(frac_ctx* c, const frac_params* params)
{
    if (!c)
        return FRAC_E_INVALID;
    std::string msg;
    if (check_params(params, msg) != FRAC_OK)
        return c->fail(FRAC_E_INVALID, msg);
    c->p = *params;
    c->dirty = true;
    return FRAC_OK;
}

static int copy_host_plane(HostPlane& hp, const uint8_t* p, uint32_t w, uint32_t h, uint32_t stride)
{
    if (!p || w == 0 || h == 0 || stride < w)
        return FRAC_E_INVALID;
    hp.w = w;
    hp.h = h;
    hp.data.resize((size_t)w * h);
    for (uint32_t y = 0; y < h; ++y)
        std::memcpy(hp.data.data() + (size_t)y * w, p + (size_t)y * stride, w);
    return FRAC_OK;
}

// A new frame of the same geometry keeps the prepared range/domain structures unless the
// classifier is on (categories depend on the pixels): without it a video frame costs the upload
// and the search only.
static void planes_changed(frac_ctx* c, uint32_t sw, uint32_t sh, uint32_t tw, uint32_t th, bool same)
{
    const bool geometry_kept = c->planes_set && c->src.w == sw && c->src.h == sh && c->tgt.w == tw &&
                               c->tgt.h == th && c->same_plane == same;
    if (!geometry_kept || c->p.use_classifier)
        c->dirty = true;
    c->src.w = sw;
    c->src.h = sh;
    c->tgt.w = tw;
    c->tgt.h = th;
    c->same_plane = same;
    c->planes_set = true;
    c->ran = false;
}

int frac_set_planes(frac_ctx* c, const uint8_t* src, uint32_t sw, uint32_t sh, uint32_t sstride, const uint8_t* tgt,
                    uint32_t tw, uint32_t th, uint32_t tstride)
{
    if (!c)
        return FRAC_E_INVALID;
    FRAC_HIP(c, hipSetDevice(c->device));
    if (!src || sw == 0 || sh == 0 || sstride < sw)
        return c->fail(FRAC_E_INVALID, "invalid source plane");
    const bool same = tgt == nullptr || tgt == src;
    if (!same && (tw == 0 || th == 0 || tstride < tw))
        return c->fail(FRAC_E_INVALID, "invalid target plane");
    FRAC_TRY(settle_fallback(c)); // the last run's fp32-regime ranges read the planes the uploads overwrite
    FRAC_TRY(upload_plane(c, src, sw, sh, sstride, c->d_src, c->d_sstride));
    if (!same)
        FRAC_TRY(upload_plane(c, tgt, tw, th, tstride, c->d_tgt, c->d_tstride));
    planes_changed(c, sw, sh, same ? sw : tw, same ? sh : th, same);
    return FRAC_OK;
}

int frac_set_frame(frac_ctx* c, const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride)
{
    return frac_set_planes(c, plane, w, h, stride, nullptr, 0, 0, 0);
}

static int set_frame_device(frac_ctx* c, const void* d_plane, uint32_t w, uint32_t h, uint32_t stride, bool wait)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!d_plane || w == 0 || h == 0 || stride < w)
        return c->fail(FRAC_E_INVALID, "invalid device plane");
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_TRY(settle_fallback(c)); // the last run's fp32-regime ranges read the plane this copy overwrites
    // the frame stays on the device: the classifier pre-pass runs there too
    c->d_sstride = (w + 63u) & ~63u;
    FRAC_HIP(c, c->d_src.ensure((size_t)c->d_sstride * (h + 1)));
    if (stride == c->d_sstride) // rows already at the device pitch: one linear copy (the 2-D path is slower)
        FRAC_HIP(c, hipMemcpyAsync(c->d_src.ptr, d_plane, (size_t)stride * (h - 1) + w, hipMemcpyDeviceToDevice,
                                   c->stream));
    else
        FRAC_HIP(c, hipMemcpy2DAsync(c->d_src.ptr, c->d_sstride, d_plane, stride, w, h, hipMemcpyDeviceToDevice,
                                     c->stream));
    if (wait)
        FRAC_HIP(c, hipStreamSynchronize(c->stream));
    planes_changed(c, w, h, w, h, true);
    return FRAC_OK;
}

int frac_set_frame_device(frac_ctx* c, const void* d_plane, uint32_t w, uint32_t h, uint32_t stride)
{
    return set_frame_device(c, d_plane, w, h, stride, true);
}

// Frame streaming from host memory: the upload runs on the context's copy stream into the plane buffer the
// current runs do not read, after the runs that last read that buffer (next_free); the context's stream waits
// for the upload (up_done) and the buffers swap, so frame k+1 crosses PCIe while frame k searches.
int frac_set_frame_async(frac_ctx* c, const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!plane || w == 0 || h == 0 || stride < w)
        return c->fail(FRAC_E_INVALID, "invalid plane");
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_TRY(settle_fallback(c)); // the last run's fp32-regime ranges read the current plane
    if (!c->copy_stream) {
        FRAC_HIP(c, hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
        FRAC_HIP(c, hipEventCreateWithFlags(&c->up_done, hipEventDisableTiming));
        FRAC_HIP(c, hipEventCreateWithFlags(&c->next_free, hipEventDisableTiming));
    }
    const uint32_t dstride = (w + 63u) & ~63u;
    if (c->d_src_next.cap < (size_t)dstride * (h + 1)) { // a (re)allocation: nothing may still read the buffer
        FRAC_HIP(c, hipStreamSynchronize(c->stream));
        FRAC_HIP(c, c->d_src_next.ensure((size_t)dstride * (h + 1)));
    }
    if (c->next_free_recorded) // the runs that read this buffer before the last swap are done
        FRAC_HIP(c, hipStreamWaitEvent(c->copy_stream, c->next_free, 0));
    if (stride == dstride)
        FRAC_HIP(c, hipMemcpyAsync(c->d_src_next.ptr, plane, (size_t)stride * (h - 1) + w, hipMemcpyHostToDevice,
                                   c->copy_stream));
    else
        FRAC_HIP(c, hipMemcpy2DAsync(c->d_src_next.ptr, dstride, plane, stride, w, h, hipMemcpyHostToDevice,
                                     c->copy_stream));
    FRAC_HIP(c, hipEventRecord(c->up_done, c->copy_stream));
    FRAC_HIP(c, hipStreamWaitEvent(c->stream, c->up_done, 0));
    std::swap(c->d_src, c->d_src_next);
    c->d_sstride = dstride;
    // the plane now in d_src_next is free once everything the context enqueued so far has run
    FRAC_HIP(c, hipEventRecord(c->next_free, c->stream));
    c->next_free_recorded = true;
    planes_changed(c, w, h, w, h, true);
    return FRAC_OK;
}

int frac_set_frame_device_async(frac_ctx* c, const void* d_plane, uint32_t w, uint32_t h, uint32_t stride)
{
    return set_frame_device(c, d_plane, w, h, stride, false);
}

int frac_set_domains(frac_ctx* c, const frac_grid_item* d, size_t nd)
{
    if (!c)
        return FRAC_E_INVALID;
    if (nd && !d)
        return c->fail(FRAC_E_INVALID, "domains is NULL");
    FRAC_TRY(check_domains(c, d, nd));
    c->doms.assign(d, d + nd);
    c->doms_set = true;
    c->doms_uploaded = false;
    c->doms_trusted = false;
    c->dirty = true;
    return FRAC_OK;
}

int frac_set_ranges(frac_ctx* c, const frac_grid_item* r, size_t nr)
{
    if (!c)
        return FRAC_E_INVALID;
    if (nr && !r)
        return c->fail(FRAC_E_INVALID, "ranges is NULL");
    c->ranges.assign(r, r + nr);
    c->ranges_set = true;
    c->ranges_dev = false;
    c->dirty = true;
    c->ran = false;
    return FRAC_OK;
}

int frac_run(frac_ctx* c)
{
    if (!c)
        return FRAC_E_INVALID;
    FRAC_HIP(c, hipSetDevice(c->device));
    {
        std::string msg;
        if (check_ab_knobs(msg) != FRAC_OK)
            return c->fail(FRAC_E_INVALID, msg);
    }
    {
        // the work lists prepare() builds depend on the A/B knobs: a change re-prepares
        int var = 0;
        FRAC_TRY(mfma_variant(c, var));
        const int knobs = var * 2 + (mfma_dft_enabled(c) ? 1 : 0);
        if (knobs != c->prep_knobs)
            c->dirty = true;
        c->prep_knobs = knobs;
    }
    // a new run owns the records: the previous run's fused-resolver state and its unsettled fallback
    // (whose saved args may name buffers prepare() is about to reallocate) go, whichever path runs next
    c->fit_fused = false;
    c->fb_pending = false;
    if (c->dirty)
        FRAC_TRY(prepare(c));
    int rc;
    switch (c->generic ? 0 : c->n) {
    case 0: rc = launch_generic(c); break;
    case 2: rc = launch_all<2>(c); break;
    case 4: rc = launch_all<4>(c); break;
    case 16: rc = launch_all<16>(c); break;
    default: rc = launch_all<8>(c); break;
    }
    const uint32_t nr = (uint32_t)nranges(c);
    if (rc == FRAC_OK && c->tuple_sink && nr) {
        if (c->fit_fused) // the resolvers wrote the tuples; the fp32-regime ranges' come with their records
            rc = settle_fallback(c);
        else // records by a separate fit: packed from them
            pack_tuples<<<(nr + 255) / 256, 256, 0, c->stream>>>(c->d_out.ptr, c->d_aux.ptr, c->d_porig.ptr, nr,
                                                                 c->tuple_sink);
    }
    if (rc == FRAC_OK)
        c->ran = true;
    return rc;
}

int frac_set_tuple_sink(frac_ctx* c, void* dst)
{
    if (!c)
        return FRAC_E_INVALID;
    c->tuple_sink = static_cast<frac_tuple*>(dst);
    return FRAC_OK;
}

int frac_sync(frac_ctx* c)
{
    if (!c)
        return FRAC_E_INVALID;
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_TRY(settle_fallback(c)); // after the sync the records are complete
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    return FRAC_OK;
}

int frac_fetch(frac_ctx* c, frac_encode_item* out, frac_stats* stats)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!c->ran)
        return c->fail(FRAC_E_STATE, "frac_fetch before frac_run");
    const size_t nr = nranges(c);
    if (nr && out)
        FRAC_HIP(c, hipMemcpyAsync(out, c->d_out.ptr, nr * sizeof(frac_encode_item), hipMemcpyDeviceToHost, c->stream));
    if (nr)
        FRAC_HIP(c, hipMemcpyAsync(c->h_aux.data(), c->d_aux.ptr, nr * sizeof(RangeAux), hipMemcpyDeviceToHost,
                                   c->stream));
    if (nr && stats && c->p.use_classifier) { // the per-range buckets of the reject count
        c->h_rkey.resize(nr);
        FRAC_HIP(c, hipMemcpyAsync(c->h_rkey.data(), c->d_rkey.ptr, nr * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   c->stream));
    }
    unsigned long long sea_count = 0;
    const bool sea_ran = c->engine_ran == FRAC_ENGINE_SEA && c->form_ran == FRAC_FORM_SEA;
    if (sea_ran)
        FRAC_HIP(c, hipMemcpyAsync(&sea_count, c->d_sea_count.ptr, sizeof(sea_count), hipMemcpyDeviceToHost,
                                   c->stream));
    uint32_t listed = 0; // the fused resolvers' fp32-regime ranges (settle_fallback)
    if (c->fb_pending)
        FRAC_HIP(c, hipMemcpyAsync(&listed, c->d_fb_count.ptr, sizeof(listed), hipMemcpyDeviceToHost, c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    if (c->fb_pending) {
        if (listed) { // rare: their records come from fallback_grid, then the copies again
            FRAC_HIP(c, hipSetDevice(c->device));
            FRAC_TRY(settle_fallback(c));
            if (nr && out)
                FRAC_HIP(c, hipMemcpyAsync(out, c->d_out.ptr, nr * sizeof(frac_encode_item), hipMemcpyDeviceToHost,
                                           c->stream));
            if (nr)
                FRAC_HIP(c, hipMemcpyAsync(c->h_aux.data(), c->d_aux.ptr, nr * sizeof(RangeAux),
                                           hipMemcpyDeviceToHost, c->stream));
            FRAC_HIP(c, hipStreamSynchronize(c->stream));
        }
        c->fb_pending = false;
    }
    if (sea_ran)
        c->evaluated_ran = sea_count;
    if (stats) {
        std::memset(stats, 0, sizeof(*stats));
        stats->total_mappings = (uint64_t)c->doms.size() * nr;
        stats->engine = c->engine_ran;
        stats->search_form = c->form_ran;
        stats->matrix_flops = c->flops_ran;
        stats->evaluated_mappings = c->evaluated_ran;
        const uint64_t nd = c->doms.size();
        if (c->p.use_classifier) { // a hit's rejects depend on its domain's grid index: the pool order
            bool any_hit = false;
            for (size_t r = 0; r < nr && !any_hit; ++r)
                any_hit = (c->h_aux[r].flags & kAuxHit) && !(c->h_aux[r].flags & kAuxEmpty);
            if (any_hit) {
                c->h_porig.resize(c->npos);
                FRAC_HIP(c, hipMemcpyAsync(c->h_porig.data(), c->d_porig.ptr, c->npos * sizeof(uint32_t),
                                           hipMemcpyDeviceToHost, c->stream));
                FRAC_HIP(c, hipStreamSynchronize(c->stream));
            }
        }
        for (size_t r = 0; r < nr; ++r) {
            const RangeAux& ax = c->h_aux[r];
            const int b = c->p.use_classifier ? (int)c->h_rkey[r] : 0;
            const uint64_t bsize = c->bucket_end[b] - c->bucket_begin[b];
            if (ax.flags & kAuxEmpty) {
                ++stats->empty_ranges;
                if (c->p.use_classifier)
                    stats->rejected_mappings += nd;
                continue;
            }
            if (ax.flags & kAuxFallback)
                ++stats->fallback_ranges;
            if (ax.flags & kAuxHit) {
                ++stats->hit_ranges;
                if (c->p.use_classifier)
                    stats->rejected_mappings += (uint64_t)c->h_porig[ax.pos] - (ax.pos - c->bucket_begin[b]);
            } else if (c->p.use_classifier) {
                stats->rejected_mappings += nd - bsize;
            }
        }
        if (c->p.flags & FRAC_FLAG_TIMING) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, last_event(c, 0), last_event(c, 3)) == hipSuccess)
                stats->ms_device = ms;
            if (hipEventElapsedTime(&ms, last_event(c, 0), last_event(c, 1)) == hipSuccess)
                stats->ms_prep = ms;
            if (hipEventElapsedTime(&ms, last_event(c, 1), last_event(c, 2)) == hipSuccess)
                stats->ms_search = ms;
            if (hipEventElapsedTime(&ms, last_event(c, 2), last_event(c, 3)) == hipSuccess)
                stats->ms_finish = ms;
        }
    }
    return FRAC_OK;
}

int frac_timing_history(frac_ctx* c, frac_run_timing* out, size_t cap, size_t* n_out)
{
    if (!c || !n_out)
        return FRAC_E_INVALID;
    *n_out = 0;
    if (!(c->p.flags & FRAC_FLAG_TIMING))
        return c->fail(FRAC_E_STATE, "timing history needs FRAC_FLAG_TIMING");
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    const uint64_t first = std::max<uint64_t>(c->hist_read, c->hist_runs > kHistRuns ? c->hist_runs - kHistRuns : 0);
    size_t k = 0;
    for (uint64_t r = first; r < c->hist_runs; ++r, ++k) {
        if (!out || k >= cap)
            continue;
        hipEvent_t* e = &c->hist[(size_t)(r % kHistRuns) * 4];
        float ms[4] = {0.f, 0.f, 0.f, 0.f};
        const int pairs[4][2] = {{0, 3}, {0, 1}, {1, 2}, {2, 3}};
        for (int q = 0; q < 4; ++q)
            if (hipEventElapsedTime(&ms[q], e[pairs[q][0]], e[pairs[q][1]]) != hipSuccess)
                ms[q] = 0.f;
        out[k] = frac_run_timing{ms[0], ms[1], ms[2], ms[3]};
    }
    (void)hipGetLastError(); // an unrecorded boundary leaves a sticky "not ready": not an error
    *n_out = k;
    if (out)
        c->hist_read = c->hist_runs;
    return FRAC_OK;
}

int frac_search(frac_ctx* c, const frac_grid_item* ranges, size_t nr, frac_encode_item* out, frac_stats* stats)
{
    FRAC_TRY(frac_set_ranges(c, ranges, nr));
    FRAC_TRY(frac_run(c));
    return frac_fetch(c, out, stats);
}

int frac_set_stream(frac_ctx* c, void* s)
{
    if (!c)
        return FRAC_E_INVALID;
    hipStream_t next = s ? reinterpret_cast<hipStream_t>(s) : c->own_stream;
    if (next == c->stream)
        return FRAC_OK;
    FRAC_HIP(c, hipSetDevice(c->device));
    // the last run's fallback goes on the stream its search and resolve ran on, and everything enqueued on
    // that stream so far comes before what is enqueued on the new one: a switch keeps the context's order
    FRAC_TRY(settle_fallback(c));
    if (!c->handoff)
        FRAC_HIP(c, hipEventCreateWithFlags(&c->handoff, hipEventDisableTiming));
    FRAC_HIP(c, hipEventRecord(c->handoff, c->stream));
    FRAC_HIP(c, hipStreamWaitEvent(next, c->handoff, 0));
    c->stream = next;
    return FRAC_OK;
}

void* frac_get_stream(frac_ctx* c) { return c ? reinterpret_cast<void*>(c->stream) : nullptr; }

const frac_encode_item* frac_device_results(frac_ctx* c)
{
    if (!c)
        return nullptr;
    // work enqueued on the context's stream after this call reads complete records
    if (c->fb_pending && (hipSetDevice(c->device) != hipSuccess || settle_fallback(c) != FRAC_OK))
        return nullptr;
    return c->d_out.ptr;
}

static int encode_quadtree_impl(frac_ctx* c, const frac_quadtree_params* qp, frac_encode_item* out,
                                frac_qt_leaf* out32, size_t cap, size_t* n_out, frac_stats* stats);

int frac_encode_quadtree(frac_ctx* c, const frac_quadtree_params* qp, frac_encode_item* out, size_t cap,
                         size_t* n_out, frac_stats* stats)
{
    return encode_quadtree_impl(c, qp, out, nullptr, cap, n_out, stats);
}

int frac_encode_quadtree_leaves(frac_ctx* c, const frac_quadtree_params* qp, frac_qt_leaf* out, size_t cap,
                                size_t* n_out, frac_stats* stats)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!qp || !n_out)
        return c->fail(FRAC_E_INVALID, "quadtree: params and n_out are required");
    if (!c->planes_set)
        return c->fail(FRAC_E_STATE, "quadtree: no frame set");
    const uint32_t W = c->src.w, H = c->src.h;
    if (W > 0xffffu || H > 0xffffu)
        return c->fail(FRAC_E_INVALID, "quadtree leaves: a frame side above 65535 does not fit the 16-bit origins");
    if (qp->min_size >= 2 && frac_uniform_grid(W, H, 2 * qp->min_size, qp->min_size, nullptr, 0) >= FRAC_QT_NO_DOMAIN)
        return c->fail(FRAC_E_INVALID, "quadtree leaves: the finest level has more domains than a 24-bit index holds");
    return encode_quadtree_impl(c, qp, nullptr, out, cap, n_out, stats);
}

// frac_encode_quadtree (out: 64-byte records) and frac_encode_quadtree_leaves (out32: 32-byte leaves)
static int encode_quadtree_impl(frac_ctx* c, const frac_quadtree_params* qp, frac_encode_item* out,
                                frac_qt_leaf* out32, size_t cap, size_t* n_out, frac_stats* stats)
{
    if (!c)
        return FRAC_E_INVALID;
    // the levels' runs write no tuples into a frac_run sink (it is sized for the context's own ranges)
    struct SinkAside {
        frac_ctx* c;
        frac_tuple* saved;
        ~SinkAside() { c->tuple_sink = saved; }
    } aside{c, c->tuple_sink};
    c->tuple_sink = nullptr;
    if (!qp || !n_out)
        return c->fail(FRAC_E_INVALID, "quadtree: params and n_out are required");
    auto valid = [](uint32_t v) { return v == 2 || v == 4 || v == 8 || v == 16; };
    if (!valid(qp->max_size) || !valid(qp->min_size) || qp->min_size > qp->max_size)
        return c->fail(FRAC_E_INVALID, "quadtree: sizes must be 2, 4, 8 or 16 with min_size <= max_size");
    if (!c->planes_set)
        return c->fail(FRAC_E_STATE, "quadtree: no frame set");
    {
        // the device-planned path never enters frac_run, so it checks the A/B knobs itself (a product
        // build refuses them here as frac_run does)
        std::string msg;
        if (check_ab_knobs(msg) != FRAC_OK)
            return c->fail(FRAC_E_INVALID, msg);
    }
    // every buffer below (ensure(), the pinned counters, the level launches) belongs to this context's
    // device, whatever device the calling thread has current
    FRAC_HIP(c, hipSetDevice(c->device));
    const uint32_t W = c->src.w, H = c->src.h;
    if (!c->same_plane && (c->tgt.w != W || c->tgt.h != H))
        return c->fail(FRAC_E_INVALID, "quadtree: source and target planes must have one size");
    auto grid = [&](uint32_t size, uint32_t off) {
        std::vector<frac_grid_item> g(frac_uniform_grid(W, H, size, off, nullptr, 0));
        if (!g.empty())
            frac_uniform_grid(W, H, size, off, g.data(), g.size());
        return g;
    };
    frac_stats total{};
    HostTrace tr("quadtree");
    if (c->qt_w != W || c->qt_h != H) {
        for (auto& g : c->qt_doms)
            g.clear();
        for (auto& v : c->qt_dvalid)
            v = false;
        c->qt_w = W;
        c->qt_h = H;
    }
    if (out32 && !qt_device_planned(c, qp)) {
        // the host-planned levels (other engines, tuning knobs): the records, then packed here
        std::vector<frac_encode_item> rec(cap);
        FRAC_TRY(encode_quadtree_impl(c, qp, cap ? rec.data() : nullptr, nullptr, cap, n_out, stats));
        const size_t m = std::min(cap, *n_out);
        for (size_t i = 0; i < m; ++i) {
            const uint32_t n = rec[i].w;
            out32[i] = qt_leaf_of(rec[i], W >= 2 * n ? (W - 2 * n) / n + 1 : 0u);
        }
        return FRAC_OK;
    }
    LevelGrid level{c, c->doms_set};
    if (qt_device_planned(c, qp))
        return qt_encode_dev(c, qp, level, out, cap, n_out, stats, out32);
    // the host-planned levels start from the first level's grid (built here only: ≈40 µs of host time
    // before the device-planned frame's first launch)
    std::vector<frac_grid_item> pending = grid(qp->max_size, qp->max_size);
    // the level-to-level step runs on the device (qt_flags, scan, qt_scatter): each level's leaves are
    // appended to d_qt_leaves and its split ranges' quadrants become the next level's device range list;
    // the host reads one count per level and the leaves once at the end
    const size_t max_leaves = (size_t)(W / qp->min_size) * (H / qp->min_size);
    FRAC_HIP(c, c->d_qt_leaves.ensure(std::max<size_t>(max_leaves, 1)));
    // the level range lists swap between d_ranges and d_qt_next: both at the worst-case size up front, so
    // no level (of this or a later frame) reallocates one (hipFree would also synchronise the device)
    FRAC_HIP(c, c->d_ranges.ensure(std::max<size_t>(max_leaves, 1)));
    FRAC_HIP(c, c->d_qt_next.ensure(std::max<size_t>(max_leaves, 1)));
    FRAC_HIP(c, c->d_qt_count.ensure(1));
    FRAC_HIP(c, c->d_qt_stats.ensure(5));
    if (stats)
        FRAC_HIP(c, hipMemsetAsync(c->d_qt_stats.ptr, 0, 5 * sizeof(unsigned long long), c->stream));
    uint32_t n_leaves = 0;
    size_t level_nr = pending.size();
    FRAC_TRY(frac_set_ranges(c, pending.data(), pending.size()));
    for (uint32_t n = qp->max_size; level_nr && n >= qp->min_size; n /= 2) {
        const int lv = __builtin_ctz(n);
        if (c->qt_doms[lv].empty())
            c->qt_doms[lv] = grid(2 * n, n);
        level.in(lv);
        c->dirty = true;
        tr.mark("grids");
        FRAC_TRY(frac_run(c));
        FRAC_TRY(settle_fallback(c)); // the level's records are complete before qt_flags reads them
        tr.mark("run (enqueue)");
        // the level's statistics accumulate on the device (no per-level download or host loop); the
        // counters are read once after the last level, the event times after this level's count
        const uint32_t nr = (uint32_t)level_nr;
        if (stats) {
            QtBuckets qb{};
            qb.nb = (uint32_t)c->bucket_begin.size();
            for (uint32_t b = 0; b < qb.nb && b < (uint32_t)kMaxBuckets; ++b) {
                qb.beg[b] = c->bucket_begin[b];
                qb.end[b] = c->bucket_end[b];
            }
            const bool sea_ran = c->engine_ran == FRAC_ENGINE_SEA && c->form_ran == FRAC_FORM_SEA;
            qt_level_stats<<<(nr + 255) / 256, 256, 0, c->stream>>>(
                c->d_aux.ptr, c->d_rkey.ptr, c->d_porig.ptr, nr, (uint64_t)c->doms.size(), c->p.use_classifier ? 1 : 0,
                qb, sea_ran ? c->d_sea_count.ptr : nullptr, c->d_qt_stats.ptr);
            total.total_mappings += (uint64_t)c->doms.size() * nr;
            total.engine = c->engine_ran;
            total.search_form = c->form_ran;
            total.matrix_flops += c->flops_ran;
            if (!sea_ran)
                total.evaluated_mappings += c->evaluated_ran;
        }
        level.out();
        tr.mark("level stats (enqueue)");
        FRAC_HIP(c, c->d_qt_flags.ensure(nr));
        FRAC_HIP(c, c->d_qt_offs.ensure(nr));
        size_t need = 0;
        FRAC_HIP(c, hipcub::DeviceScan::ExclusiveSum(nullptr, need, c->d_qt_flags.ptr, c->d_qt_offs.ptr, (int)nr,
                                                     c->stream));
        if (need > c->qt_tmp_bytes) {
            FRAC_HIP(c, c->d_qt_tmp.ensure(need));
            c->qt_tmp_bytes = need;
        }
        qt_flags<<<(nr + 255) / 256, 256, 0, c->stream>>>(c->d_out.ptr, nr, n > qp->min_size ? 1 : 0,
                                                         qp->split_distance, c->d_qt_flags.ptr);
        size_t tb = c->qt_tmp_bytes;
        FRAC_HIP(c, hipcub::DeviceScan::ExclusiveSum(c->d_qt_tmp.ptr, tb, c->d_qt_flags.ptr, c->d_qt_offs.ptr, (int)nr,
                                                     c->stream));
        // d_qt_next holds max_leaves items already: the 4·nsplit quadrants tile part of the plane at
        // ≥ min_size each, and the last level (n == min_size) splits nothing
        qt_scatter<<<(nr + 255) / 256, 256, 0, c->stream>>>(c->d_out.ptr, c->d_ranges.ptr, nr, c->d_qt_flags.ptr,
                                                           c->d_qt_offs.ptr, c->d_qt_leaves.ptr, n_leaves,
                                                           c->d_qt_next.ptr, c->d_qt_count.ptr);
        uint32_t nsplit = 0;
        FRAC_HIP(c, hipMemcpyAsync(&nsplit, c->d_qt_count.ptr, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
        FRAC_HIP(c, hipStreamSynchronize(c->stream));
        if (stats && (c->p.flags & FRAC_FLAG_TIMING)) { // the level's run has completed
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, last_event(c, 0), last_event(c, 3)) == hipSuccess)
                total.ms_device += ms;
            if (hipEventElapsedTime(&ms, last_event(c, 0), last_event(c, 1)) == hipSuccess)
                total.ms_prep += ms;
            if (hipEventElapsedTime(&ms, last_event(c, 1), last_event(c, 2)) == hipSuccess)
                total.ms_search += ms;
            if (hipEventElapsedTime(&ms, last_event(c, 2), last_event(c, 3)) == hipSuccess)
                total.ms_finish += ms;
        }
        n_leaves += nr - nsplit;
        level_nr = 4 * (size_t)nsplit;
        // the next level searches the device-built quadrants
        std::swap(c->d_ranges, c->d_qt_next);
        c->ranges_dev = true;
        c->nr_dev = (uint32_t)level_nr;
        c->n_dev = n / 2;
        c->ranges_set = true;
        c->ran = false;
        tr.mark("split (device)");
    }
    c->ranges_dev = false;
    c->ranges.clear();
    c->dirty = true;
    c->ran = false;
    *n_out = n_leaves;
    if (out && n_leaves)
        FRAC_HIP(c, hipMemcpy(out, c->d_qt_leaves.ptr, std::min<size_t>(cap, n_leaves) * sizeof(frac_encode_item),
                              hipMemcpyDeviceToHost));
    tr.mark("leaves D2H");
    if (stats) {
        unsigned long long acc[5] = {0ull, 0ull, 0ull, 0ull, 0ull};
        FRAC_HIP(c, hipMemcpy(acc, c->d_qt_stats.ptr, sizeof(acc), hipMemcpyDeviceToHost));
        total.rejected_mappings = acc[0];
        total.hit_ranges = acc[1];
        total.fallback_ranges = acc[2];
        total.empty_ranges = acc[3];
        total.evaluated_mappings += acc[4];
        *stats = total;
    }
    return FRAC_OK;
}

int frac_classify_items(frac_ctx* c, frac_grid_item* items, size_t n, int target_plane)
{
    if (!c)
        return FRAC_E_INVALID;
    if (n && !items)
        return c->fail(FRAC_E_INVALID, "classify: items is NULL");
    if (!c->planes_set)
        return c->fail(FRAC_E_STATE, "classify: no frame set");
    const bool tgt = target_plane != 0 && !c->same_plane;
    const HostPlane& hp = tgt ? c->tgt : c->src;
    std::vector<frac_grid_item> v(items, items + n);
    std::vector<uint32_t> list(n);
    for (size_t i = 0; i < n; ++i) {
        if ((uint64_t)v[i].x + v[i].w > hp.w || (uint64_t)v[i].y + v[i].h > hp.h)
            return c->fail(FRAC_E_INVALID, "classify: item outside the plane");
        list[i] = (uint32_t)i;
    }
    FRAC_HIP(c, hipSetDevice(c->device));
    std::vector<int32_t> cat;
    FRAC_TRY(classify_on_device(c, v, list, tgt ? c->d_tgt.ptr : c->d_src.ptr, tgt ? c->d_tstride : c->d_sstride,
                                cat));
    for (size_t i = 0; i < n; ++i)
        items[i].category = cat[i];
    return FRAC_OK;
}

int frac_rgb_to_yuv_device(frac_ctx* c, const void* d_rgb, uint32_t w, uint32_t h, uint32_t rgb_stride, void* d_y,
                           uint32_t y_stride, void* d_u, uint32_t u_stride, void* d_v, uint32_t v_stride)
{
    if (!c)
        return FRAC_E_INVALID;
    if (w == 0 || h == 0)
        return FRAC_OK;
    if (!d_rgb || !d_y || ((w >= 2 && h >= 2) && (!d_u || !d_v)) || rgb_stride < 3ull * w || y_stride < w ||
        (w >= 2 && h >= 2 && (u_stride < w / 2 || v_stride < w / 2)))
        return c->fail(FRAC_E_INVALID, "rgb_to_yuv: invalid plane pointers or strides");
    FRAC_HIP(c, hipSetDevice(c->device));
    ColorArgs a;
    a.rgb = static_cast<const uint8_t*>(d_rgb);
    a.w = w;
    a.h = h;
    a.rgb_stride = rgb_stride;
    a.y = static_cast<uint8_t*>(d_y);
    a.ys = y_stride;
    a.u = static_cast<uint8_t*>(d_u);
    a.us = u_stride;
    a.v = static_cast<uint8_t*>(d_v);
    a.vs = v_stride;
    if (color_fast_path(a)) {
        const size_t n = (size_t)(w / 4) * (h / 2);
        rgb2yuv_quads4<<<(unsigned)((n + 255) / 256), 256, 0, c->stream>>>(a);
    } else {
        const size_t n = (size_t)((w + 1) / 2) * ((h + 1) / 2);
        rgb2yuv_generic<<<(unsigned)((n + 255) / 256), 256, 0, c->stream>>>(a);
    }
    FRAC_HIP(c, hipGetLastError());
    return FRAC_OK;
}

int frac_rgb_to_yuv(frac_ctx* c, const uint8_t* rgb, uint32_t w, uint32_t h, uint32_t rgb_stride, uint8_t* y,
                    uint8_t* u, uint8_t* v)
{
    if (!c)
        return FRAC_E_INVALID;
    if (w == 0 || h == 0)
        return FRAC_OK;
    if (!rgb || !y || (w >= 2 && h >= 2 && (!u || !v)) || rgb_stride < 3ull * w)
        return c->fail(FRAC_E_INVALID, "rgb_to_yuv: invalid buffers");
    FRAC_HIP(c, hipSetDevice(c->device));
    const uint32_t cw = w / 2, ch = h / 2;
    const uint32_t ys = (w + 63u) & ~63u, cs = (cw + 63u) & ~63u;
    const size_t rgb_bytes = (size_t)rgb_stride * h, y_bytes = (size_t)ys * h, c_bytes = (size_t)cs * std::max(ch, 1u);
    FRAC_HIP(c, c->d_color.ensure(rgb_bytes + y_bytes + 2 * c_bytes));
    uint8_t* d_rgb = c->d_color.ptr;
    uint8_t* d_y = d_rgb + rgb_bytes;
    uint8_t* d_u = d_y + y_bytes;
    uint8_t* d_v = d_u + c_bytes;
    FRAC_HIP(c, hipMemcpyAsync(d_rgb, rgb, rgb_bytes, hipMemcpyHostToDevice, c->stream));
    FRAC_TRY(frac_rgb_to_yuv_device(c, d_rgb, w, h, rgb_stride, d_y, ys, d_u, cs, d_v, cs));
    FRAC_HIP(c, hipMemcpy2DAsync(y, w, d_y, ys, w, h, hipMemcpyDeviceToHost, c->stream));
    if (cw && ch) {
        FRAC_HIP(c, hipMemcpy2DAsync(u, cw, d_u, cs, cw, ch, hipMemcpyDeviceToHost, c->stream));
        FRAC_HIP(c, hipMemcpy2DAsync(v, cw, d_v, cs, cw, ch, hipMemcpyDeviceToHost, c->stream));
    }
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    return FRAC_OK;
}

// Do the items (x, y, w, h) cover the w×h plane exactly once?  Checked on a bitmap of cells of
// the smallest item size (every item a multiple of it, aligned), so O(cells), not O(pixels).
static bool covers_exactly(const std::vector<frac_grid_item>& rects, uint32_t w, uint32_t h)
{
    if (rects.empty())
        return false;
    uint32_t g = ~0u;
    for (const auto& r : rects) {
        if (r.w == 0 || r.w != r.h)
            return false;
        g = std::min(g, r.w);
    }
    if (w % g || h % g)
        return false;
    const uint32_t cw = w / g, ch = h / g;
    std::vector<uint8_t> cell((size_t)cw * ch, 0);
    size_t covered = 0;
    for (const auto& r : rects) {
        if (r.x % g || r.y % g || r.w % g || (uint64_t)r.x + r.w > w || (uint64_t)r.y + r.h > h)
            return false;
        for (uint32_t y = r.y / g; y < (r.y + r.h) / g; ++y)
            for (uint32_t x = r.x / g; x < (r.x + r.w) / g; ++x) {
                if (cell[(size_t)y * cw + x]++)
                    return false;
                ++covered;
            }
    }
    return covered == cell.size();
}

// Fused decode (fracenc_decode.hip decode_fused / decode_check): the items tile the plane.
static int decode_fused_impl(frac_ctx* c, const frac_encode_item* d_items, size_t n, uint32_t w, uint32_t h,
                             int iters, double eps, uint8_t* plane, int* iterations, double* rms)
{
    const uint32_t stride = (w + 63u) & ~63u;
    const size_t bytes = (size_t)stride * (h + 1);
    FRAC_HIP(c, c->d_dec_src.ensure(bytes));
    FRAC_HIP(c, c->d_dec_tgt.ensure(bytes));
    const uint32_t nblk = (uint32_t)((n + 3) / 4);
    FRAC_HIP(c, c->d_dec_part.ensure(kDecodeSlots));
    FRAC_HIP(c, hipMemsetAsync(c->d_dec_part.ptr, 0, kDecodeSlots * sizeof(unsigned long long), c->stream));
    FRAC_HIP(c, c->d_dec_state.ensure(1));
    if (!c->h_dec_state)
        FRAC_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_dec_state), sizeof(DecodeState)));
    uint8_t* buf[2] = {c->d_dec_src.ptr, c->d_dec_tgt.ptr};
    FRAC_HIP(c, hipMemsetAsync(buf[0], 100, bytes, c->stream)); // Decoder2: source filled with 100
    FRAC_HIP(c, hipMemsetAsync(buf[1], 0, bytes, c->stream));
    FRAC_HIP(c, hipMemcpy2DAsync(buf[1], stride, plane, w, w, h, hipMemcpyHostToDevice, c->stream));
    FRAC_HIP(c, hipMemsetAsync(c->d_dec_state.ptr, 0, sizeof(DecodeState), c->stream));
    DecodeArgs a;
    a.stride = stride;
    a.items = d_items;
    a.n = (uint32_t)n;
    constexpr int kChunk = 8; // iterations enqueued between host checks of the convergence flag
    int enq = 0;
    while (enq < iters) {
        const int stop = std::min(iters, enq + kChunk);
        for (; enq < stop; ++enq) {
            a.src = buf[enq & 1];
            a.tgt = buf[(enq + 1) & 1];
            decode_fused<<<nblk, 256, 0, c->stream>>>(a, c->d_dec_state.ptr, c->d_dec_part.ptr);
            decode_check<<<1, kDecodeSlots, 0, c->stream>>>(c->d_dec_part.ptr, (uint64_t)w * h, eps, enq, iters - 1,
                                                            c->d_dec_state.ptr);
        }
        FRAC_HIP(c, hipMemcpyAsync(c->h_dec_state, c->d_dec_state.ptr, sizeof(DecodeState), hipMemcpyDeviceToHost,
                                   c->stream));
        FRAC_HIP(c, hipStreamSynchronize(c->stream));
        if (c->h_dec_state->done)
            break;
    }
    int it = 0;
    double r = 0.0;
    if (iters > 0) {
        it = c->h_dec_state->iterations;
        r = c->h_dec_state->rms;
    }
    // the final target: step `it` when the loop broke there, else step iters − 1
    const int last = iters > 0 ? (c->h_dec_state->done ? it : iters - 1) : -1;
    const uint8_t* fin = last >= 0 ? buf[(last + 1) & 1] : buf[1];
    FRAC_HIP(c, hipMemcpy2DAsync(plane, w, fin, stride, w, h, hipMemcpyDeviceToHost, c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    FRAC_HIP(c, hipGetLastError());
    if (iterations)
        *iterations = it;
    if (rms)
        *rms = r;
    return FRAC_OK;
}

static int decode_impl(frac_ctx* c, const frac_encode_item* d_items, size_t n, uint32_t w, uint32_t h, int max_iter,
                       double eps, uint8_t* plane, int* iterations, double* rms, bool fused = false)
{
    if (!plane || w == 0 || h == 0)
        return c->fail(FRAC_E_INVALID, "decode: invalid plane");
    {
        std::string msg;
        if (check_ab_knobs(msg) != FRAC_OK)
            return c->fail(FRAC_E_INVALID, msg);
    }
    if (fused &&!(c->p.flags & FRAC_FLAG_DECODE_STEPWISE) && ab_knob("FRAC_DECODE_UNFUSED") == nullptr)
        return decode_fused_impl(c, d_items, n, w, h, max_iter < 0 ? 300 : max_iter, eps, plane, iterations, rms);
    const uint32_t stride = (w + 63u) & ~63u;
    const size_t bytes = (size_t)stride * (h + 1);
    FRAC_HIP(c, c->d_dec_src.ensure(bytes));
    FRAC_HIP(c, c->d_dec_tgt.ensure(bytes));
    FRAC_HIP(c, c->d_dec_sum.ensure(1));
    if (!c->h_dec_sum)
        FRAC_HIP(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_dec_sum), sizeof(unsigned long long)));
    // Decoder2::decode: source filled with 100, target = the caller's plane
    FRAC_HIP(c, hipMemsetAsync(c->d_dec_src.ptr, 100, bytes, c->stream));
    FRAC_HIP(c, hipMemsetAsync(c->d_dec_tgt.ptr, 0, bytes, c->stream));
    FRAC_HIP(c, hipMemcpy2DAsync(c->d_dec_tgt.ptr, stride, plane, w, w, h, hipMemcpyHostToDevice, c->stream));
    const int iters = max_iter < 0 ? 300 : max_iter;
    DecodeArgs a;
    a.src = c->d_dec_src.ptr;
    a.tgt = c->d_dec_tgt.ptr;
    a.stride = stride;
    a.items = d_items;
    a.n = (uint32_t)n;
    const uint32_t rms_blocks = (uint32_t)std::min<size_t>(1024, ((size_t)w * h + 255) / 256);
    int i = 0;
    double r = 0.0;
    for (; i < iters; ++i) {
        if (n)
            decode_apply<<<(unsigned)((n + 3) / 4), 256, 0, c->stream>>>(a);
        FRAC_HIP(c, hipMemsetAsync(c->d_dec_sum.ptr, 0, sizeof(unsigned long long), c->stream));
        decode_rms<<<rms_blocks, 256, 0, c->stream>>>(c->d_dec_src.ptr, c->d_dec_tgt.ptr, w, h, stride, c->d_dec_sum.ptr);
        FRAC_HIP(c, hipMemcpyAsync(c->h_dec_sum, c->d_dec_sum.ptr, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                                   c->stream));
        FRAC_HIP(c, hipStreamSynchronize(c->stream));
        // the reference accumulates in int32 (metrics.h:29): reproduce its wrap-around
        const int32_t s32 = (int32_t)(uint32_t)(*c->h_dec_sum & 0xffffffffull);
        r = (double)s32 / (double)((uint64_t)w * h);
        if (r < eps)
            break;
        FRAC_HIP(c, hipMemcpyAsync(c->d_dec_src.ptr, c->d_dec_tgt.ptr, bytes, hipMemcpyDeviceToDevice, c->stream));
    }
    FRAC_HIP(c, hipMemcpy2DAsync(plane, w, c->d_dec_tgt.ptr, stride, w, h, hipMemcpyDeviceToHost, c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    FRAC_HIP(c, hipGetLastError());
    if (iterations)
        *iterations = i;
    if (rms)
        *rms = r;
    return FRAC_OK;
}

int frac_decode(frac_ctx* c, const frac_encode_item* items, size_t n, uint32_t w, uint32_t h, int max_iter,
                double rms_eps, uint8_t* plane, int* iterations, double* rms)
{
    if (!c)
        return FRAC_E_INVALID;
    if (n && !items)
        return c->fail(FRAC_E_INVALID, "decode: items is NULL");
    for (size_t i = 0; i < n; ++i) {
        const frac_encode_item& e = items[i];
        if ((uint64_t)e.x + e.w > w || (uint64_t)e.y + e.h > h || e.match.score.transform < 0 ||
            e.match.score.transform > 7 ||
            (e.match.sw && ((uint64_t)e.match.x + e.match.sw > w || (uint64_t)e.match.y + e.match.sh > h)))
            return c->fail(FRAC_E_INVALID, "decode: item outside the plane or bad transform");
        // a rectangular (or degenerate) domain: the transformed 2×2 samples (Frac::copy's fit points,
        // DecodeUtils.hpp:9-25) may leave the patch; they must stay inside the plane
        if (e.match.sw && (e.match.sw != e.match.sh || e.match.sw < 2) &&
            (e.match.sw < 2 || e.match.sh < 2 || e.w == 0 || e.h == 0 ||
             !box_inside(sample_box(e.match.score.transform, (int)e.match.sw, (int)e.match.sh, (int)e.w, (int)e.h,
                                    false, true),
                         e.match.x, e.match.y, w, h)))
            return c->fail(FRAC_E_INVALID, "decode: a transformed sample of item " + std::to_string(i) +
                                               " falls outside the plane");
    }
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_HIP(c, c->d_dec_items.ensure(n));
    if (n)
        FRAC_HIP(c, hipMemcpyAsync(c->d_dec_items.ptr, items, n * sizeof(frac_encode_item), hipMemcpyHostToDevice,
                                   c->stream));
    std::vector<frac_grid_item> rects(n);
    bool all_domains = true;
    for (size_t i = 0; i < n; ++i) {
        rects[i] = frac_grid_item{items[i].x, items[i].y, items[i].w, items[i].h, -1};
        all_domains = all_domains && items[i].match.sw != 0 && items[i].match.sh != 0;
    }
    const bool fused = all_domains && covers_exactly(rects, w, h);
    return decode_impl(c, c->d_dec_items.ptr, n, w, h, max_iter, rms_eps, plane, iterations, rms, fused);
}

int frac_decode_results(frac_ctx* c, uint32_t w, uint32_t h, int max_iter, double rms_eps, uint8_t* plane,
                        int* iterations, double* rms)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!c->ran)
        return c->fail(FRAC_E_STATE, "decode: frac_run has not been called");
    if (c->src.w > w || c->src.h > h || c->tgt.w > w || c->tgt.h > h)
        return c->fail(FRAC_E_INVALID, "decode: plane smaller than the encoded planes");
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_TRY(settle_fallback(c));
    // the fused form needs every range written: no empty (domain-less) record among the results
    bool fused = covers_exactly(c->ranges, w, h);
    if (fused && !c->ranges.empty()) {
        c->h_aux.resize(nranges(c));
        FRAC_HIP(c, hipMemcpyAsync(c->h_aux.data(), c->d_aux.ptr, nranges(c) * sizeof(RangeAux),
                                   hipMemcpyDeviceToHost, c->stream));
        FRAC_HIP(c, hipStreamSynchronize(c->stream));
        for (const RangeAux& x : c->h_aux)
            if (x.flags & kAuxEmpty) {
                fused = false;
                break;
            }
    }
    return decode_impl(c, c->d_out.ptr, nranges(c), w, h, max_iter, rms_eps, plane, iterations, rms, fused);
}

int frac_copy_tuples_device(frac_ctx* c, void* d_dst)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!c->ran)
        return c->fail(FRAC_E_STATE, "no results: frac_run has not been called");
    const uint32_t nr = (uint32_t)nranges(c);
    if (nr) {
        if (!d_dst)
            return c->fail(FRAC_E_INVALID, "copy_tuples: NULL destination");
        FRAC_HIP(c, hipSetDevice(c->device));
        FRAC_TRY(settle_fallback(c));
        pack_tuples<<<(nr + 255) / 256, 256, 0, c->stream>>>(c->d_out.ptr, c->d_aux.ptr, c->d_porig.ptr, nr,
                                                             static_cast<frac_tuple*>(d_dst));
        FRAC_HIP(c, hipGetLastError());
    }
    return FRAC_OK;
}

int frac_pack_frc1(frac_ctx* c, uint32_t cbits, uint32_t bbits, uint8_t* out, size_t cap, size_t* n_out)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!n_out)
        return c->fail(FRAC_E_INVALID, "pack_frc1: n_out is NULL");
    if (!c->ran)
        return c->fail(FRAC_E_STATE, "pack_frc1: frac_run has not been called");
    if (cbits < 2 || cbits > 16 || bbits < 2 || bbits > 16)
        return c->fail(FRAC_E_INVALID, "pack_frc1: contrast/brightness bits must be in [2, 16]");
    const uint32_t W = c->tgt.w, H = c->tgt.h, n = (uint32_t)c->n;
    if (c->src.w != W || c->src.h != H)
        return c->fail(FRAC_E_INVALID, "pack_frc1: source and target planes must have one size");
    // the stream's implicit geometry: createUniformGrid ranges (row-major) and domains
    // (compared item by item against the closed-form lattice, without building it: at C3 the two grids
    // hold 0.5 M items)
    auto same_grid = [&](const std::vector<frac_grid_item>& g, uint32_t size, uint32_t off) {
        const size_t cnt = frac_uniform_grid(W, H, size, off, nullptr, 0);
        if (cnt != g.size())
            return false;
        if (!cnt)
            return true;
        const size_t cols = (W - size) / off + 1;
        const frac_grid_item* it = g.data();
        for (size_t r = 0, k = 0; k < cnt; ++r)
            for (size_t q = 0; q < cols; ++q, ++k, ++it)
                if (it->x != q * off || it->y != r * off || it->w != size || it->h != size)
                    return false;
        return true;
    };
    if (n == 0)
        return c->fail(FRAC_E_INVALID, "pack_frc1: the stream holds square items only");
    if (!same_grid(c->ranges, n, n))
        return c->fail(FRAC_E_INVALID, "pack_frc1: ranges are not the row-major range grid");
    if (!same_grid(c->doms, 2 * n, n))
        return c->fail(FRAC_E_INVALID, "pack_frc1: domains are not the domain lattice (size 2n, stride n)");
    const uint32_t nr = (uint32_t)nranges(c), nd = (uint32_t)c->doms.size(), T = c->p.transforms;
    auto bitlen = [](uint64_t v) { uint32_t b = 0; while (v) { ++b; v >>= 1; } return b; };
    const uint32_t ib = std::max(1u, bitlen(nd)), tb = std::max(1u, bitlen(T - 1));
    const uint32_t width = ib + tb + cbits + bbits;
    if (width > 64)
        return c->fail(FRAC_E_INVALID, "pack_frc1: record wider than 64 bits");
    const uint64_t body = ((uint64_t)nr * width + 7) / 8, nwords = ((uint64_t)nr * width + 31) / 32;
    *n_out = FRAC_FRC1_HEADER_BYTES + body;
    if (!out)
        return FRAC_OK;
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_TRY(settle_fallback(c));
    Frc1MinMax mm{~0ull, 0ull, ~0ull, 0ull};
    std::vector<uint32_t> words(nwords);
    if (nr) {
        FRAC_HIP(c, c->d_frc_mm.ensure(1));
        FRAC_HIP(c, c->d_frc_rec.ensure(nr));
        FRAC_HIP(c, c->d_frc_words.ensure(nwords));
        FRAC_HIP(c, hipMemsetAsync(c->d_frc_mm.ptr, 0xff, sizeof(unsigned long long), c->stream));
        FRAC_HIP(c, hipMemsetAsync(&c->d_frc_mm.ptr->cmax, 0, sizeof(unsigned long long), c->stream));
        FRAC_HIP(c, hipMemsetAsync(&c->d_frc_mm.ptr->bmin, 0xff, sizeof(unsigned long long), c->stream));
        FRAC_HIP(c, hipMemsetAsync(&c->d_frc_mm.ptr->bmax, 0, sizeof(unsigned long long), c->stream));
        frc1_minmax<<<std::min<uint32_t>(1024, (nr + 255) / 256), 256, 0, c->stream>>>(c->d_out.ptr, nr,
                                                                                          c->d_frc_mm.ptr);
        Frc1Args a;
        a.out = c->d_out.ptr;
        a.n = nr;
        a.dstride = n;
        a.dcols = (uint32_t)((W - 2 * n) / n + 1);
        a.ndomains = nd;
        a.index_bits = ib;
        a.t_bits = tb;
        a.c_bits = cbits;
        a.b_bits = bbits;
        a.mm = c->d_frc_mm.ptr;
        a.rec = c->d_frc_rec.ptr;
        frc1_records<<<(nr + 255) / 256, 256, 0, c->stream>>>(a);
        frc1_words<<<(unsigned)((nwords + 255) / 256), 256, 0, c->stream>>>(c->d_frc_rec.ptr, nr, width, nwords,
                                                                             c->d_frc_words.ptr);
        FRAC_HIP(c, hipGetLastError());
        FRAC_HIP(c, hipMemcpyAsync(&mm, c->d_frc_mm.ptr, sizeof(mm), hipMemcpyDeviceToHost, c->stream));
        FRAC_HIP(c, hipMemcpyAsync(words.data(), c->d_frc_words.ptr, nwords * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   c->stream));
        FRAC_HIP(c, hipStreamSynchronize(c->stream));
    }
    // header "<4sHHIIIIIBBBBIIdddd" (fractencode_amd/codec.py)
    uint8_t hdr[FRAC_FRC1_HEADER_BYTES] = {};
    size_t o = 0;
    auto put = [&](const void* v, size_t k) { std::memcpy(hdr + o, v, k); o += k; };
    const uint16_t version = 1, flags = c->p.use_classifier ? 1 : 0;
    const uint32_t u32s[5] = {W, H, n, 2 * n, n};
    const uint8_t u8s[4] = {(uint8_t)T, (uint8_t)cbits, (uint8_t)bbits, (uint8_t)ib};
    const uint32_t counts[2] = {nr, nd};
    const double mm_d[4] = {nr ? dkey_inv(mm.cmin) : 0.0, nr ? dkey_inv(mm.cmax) : 0.0, nr ? dkey_inv(mm.bmin) : 0.0,
                            nr ? dkey_inv(mm.bmax) : 0.0};
    put("FRC1", 4);
    put(&version, 2);
    put(&flags, 2);
    put(u32s, sizeof(u32s));
    put(u8s, sizeof(u8s));
    put(counts, sizeof(counts));
    put(mm_d, sizeof(mm_d));
    const size_t total = FRAC_FRC1_HEADER_BYTES + body;
    std::memcpy(out, hdr, std::min<size_t>(cap, FRAC_FRC1_HEADER_BYTES));
    if (cap > FRAC_FRC1_HEADER_BYTES)
        std::memcpy(out + FRAC_FRC1_HEADER_BYTES, words.data(), std::min<size_t>(cap, total) - FRAC_FRC1_HEADER_BYTES);
    return FRAC_OK;
}

int frac_fetch_tuples(frac_ctx* c, frac_tuple* out)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!c->ran)
        return c->fail(FRAC_E_STATE, "no results: frac_run has not been called");
    const size_t nr = nranges(c);
    if (!nr)
        return FRAC_OK;
    if (!out)
        return c->fail(FRAC_E_INVALID, "fetch_tuples: NULL destination");
    FRAC_HIP(c, c->d_tuples.ensure(nr));
    FRAC_TRY(frac_copy_tuples_device(c, c->d_tuples.ptr));
    FRAC_HIP(c, hipMemcpyAsync(out, c->d_tuples.ptr, nr * sizeof(frac_tuple), hipMemcpyDeviceToHost, c->stream));
    FRAC_HIP(c, hipStreamSynchronize(c->stream));
    return FRAC_OK;
}

int frac_copy_results_device(frac_ctx* c, void* d_dst)
{
    if (!c)
        return FRAC_E_INVALID;
    if (!c->ran)
        return c->fail(FRAC_E_STATE, "no results: frac_run has not been called");
    const size_t nr = nranges(c);
    FRAC_HIP(c, hipSetDevice(c->device));
    FRAC_TRY(settle_fallback(c));
    if (nr)
        FRAC_HIP(c, hipMemcpyAsync(d_dst, c->d_out.ptr, nr * sizeof(frac_encode_item), hipMemcpyDeviceToDevice,
                                   c->stream));
    return FRAC_OK;
}

size_t frac_uniform_grid2(uint32_t W, uint32_t H, uint32_t size_w, uint32_t size_h, uint32_t off_x, uint32_t off_y,
                          frac_grid_item* out, size_t cap)
{
    // createUniformGrid's loop (image/partition2.hpp:123-133): x advances by the offset's x, a row
    // ends when the next item would cross the right edge, the grid when the next row would cross
    // the bottom edge
    // — so a row holds ⌊(W − w)/off_x⌋ + 1 items and the grid ⌊(H − h)/off_y⌋ + 1 rows (the count in closed
    // form: the loop took 0.2 ms for the 4-pixel quadtree level's domains at 2048², on every quadtree call)
    if (size_w == 0 || size_h == 0 || off_x == 0 || off_y == 0 || W < size_w || H < size_h)
        return 0;
    const size_t cols = (W - size_w) / off_x + 1, rows = (H - size_h) / off_y + 1;
    if (out) {
        size_t n = 0;
        for (size_t r = 0; r < rows && n < cap; ++r)
            for (size_t k = 0; k < cols && n < cap; ++k)
                out[n++] = frac_grid_item{(uint32_t)(k * off_x), (uint32_t)(r * off_y), size_w, size_h, -1};
    }
    return cols * rows;
}

size_t frac_uniform_grid(uint32_t W, uint32_t H, uint32_t size, uint32_t offset, frac_grid_item* out, size_t cap)
{
    return frac_uniform_grid2(W, H, size, size, offset, offset, out, cap);
}

int frac_classify(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride, frac_grid_item* items, size_t n)
{
    HostPlane hp;
    if (copy_host_plane(hp, plane, w, h, stride) != FRAC_OK || (n && !items)) {
        g_last_error = "frac_classify: invalid arguments";
        return FRAC_E_INVALID;
    }
    for (size_t i = 0; i < n; ++i) {
        if ((uint64_t)items[i].x + items[i].w > w || (uint64_t)items[i].y + items[i].h > h) {
            g_last_error = "frac_classify: item outside the plane";
            return FRAC_E_INVALID;
        }
        items[i].category = category(hp, items[i]);
    }
    return FRAC_OK;
}

int frac_transform_index(uint32_t n, uint32_t t, uint32_t pix)
{
    if (t > 7 || pix >= n * n)
        return -1;
    switch (n) {
    case 2: return fwd_index<2>((int)t, (int)pix);
    case 4: return fwd_index<4>((int)t, (int)pix);
    case 8: return fwd_index<8>((int)t, (int)pix);
    case 16: return fwd_index<16>((int)t, (int)pix);
    default: return -1;
    }
}

int64_t frac_hit_limit(double rms_threshold, uint32_t n) { return compute_hit_limit(rms_threshold, 4u * n * n); }

} // extern "C"

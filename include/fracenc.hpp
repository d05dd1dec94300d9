// fracenc.hpp — C++17 host layer over the C ABI (include/fracenc.h).
//
// The reference's host side is C++ (encode/Encoder2.hpp, encode/EncodingEngine2.hpp); this
// header gives a C++ caller the same roles without any reference types:
//
//   Engine              RAII frac_ctx: one search context on one GPU (an AbstractEncodingEngine2
//                       that takes batches, encode/EncodingEngine2.hpp:50-85)
//   EncodingEngineCore  EncodingEngineCore2's role (encode/EncodingEngine2.hpp:118-171): a host
//                       pool of engines (one std::thread each, any mix of devices) claiming
//                       BATCHES of ranges from a shared counter instead of one item at a time
//                       (:131-140); results come back in range order (the reference's order is
//                       thread-dependent, :165-168)
//   Quantizer<T>        Frac::Quantizer (encode/Quantizer.hpp:7-45) as the built reference
//                       computes it (value() with the FMA the compiler contracts)
//   createUniformGrid / preclassify / encodeQuadtree / decode   — the C ABI entry points
//   Engine's ABI 8/9 methods: an external HIP stream (void*), the tuple sink and 32-byte tuples,
//                       frame streaming (setFrameAsync / setFrameDeviceAsync), 32-byte quadtree
//                       leaves, per-run device times
//
// Errors throw fracenc::Error carrying frac_last_error.
#pragma once

#include "fracenc.h"

#include <atomic>
#include <cassert>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace fracenc {

class Error : public std::runtime_error {
public:
    explicit Error(const std::string& m) : std::runtime_error(m) {}
};

struct Params {
    uint32_t transforms = 4;    // 4: TransformMatcher::match (transformmatcher.h:41-45); 8: all dihedral
    bool use_classifier = false;
    double rms_threshold = 0.0; // encode_parameters_t::rmsThreshold
    double s_max = -1.0;        // encode_parameters_t::sMax
    uint32_t engine = FRAC_ENGINE_AUTO;
    bool timing = false;

    frac_params c() const
    {
        frac_params p{};
        p.transforms = transforms;
        p.use_classifier = use_classifier ? 1 : 0;
        p.rms_threshold = rms_threshold;
        p.s_max = s_max;
        p.engine = engine;
        p.flags = timing ? FRAC_FLAG_TIMING : 0u;
        return p;
    }
};

inline std::vector<frac_grid_item> createUniformGrid(uint32_t w, uint32_t h, uint32_t size, uint32_t offset)
{
    std::vector<frac_grid_item> g(frac_uniform_grid(w, h, size, offset, nullptr, 0));
    if (!g.empty())
        frac_uniform_grid(w, h, size, offset, g.data(), g.size());
    return g;
}

// BrightnessBlocksClassifier2::preclassify on the host (main.cpp:155-162)
inline void preclassify(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride,
                        std::vector<frac_grid_item>& items)
{
    if (frac_classify(plane, w, h, stride, items.data(), items.size()) != FRAC_OK)
        throw Error(frac_last_error(nullptr));
}

class Engine {
public:
    Engine(int device, const Params& p)
    {
        const frac_params cp = p.c();
        ctx_ = frac_create(device, &cp);
        if (!ctx_)
            throw Error(std::string("frac_create: ") + frac_last_error(nullptr));
    }
    ~Engine() { frac_destroy(ctx_); }
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;
    Engine(Engine&& o) noexcept : ctx_(std::exchange(o.ctx_, nullptr)), w_(o.w_), h_(o.h_) {}

    frac_ctx* get() const { return ctx_; }

    void setFrame(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride)
    {
        check(frac_set_frame(ctx_, plane, w, h, stride));
        w_ = w;
        h_ = h;
    }
    void setFrameDevice(const void* d_plane, uint32_t w, uint32_t h, uint32_t stride)
    {
        check(frac_set_frame_device(ctx_, d_plane, w, h, stride));
        w_ = w;
        h_ = h;
    }
    // ABI 9: frame streaming.  setFrameAsync uploads on the context's copy stream into its second plane buffer
    // while the runs already enqueued read the current one (pinned host memory makes it asynchronous; the plane
    // must stay unchanged until a later sync / fetch); setFrameDeviceAsync copies a device plane on the
    // context's stream without a host wait.
    void setFrameAsync(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride)
    {
        check(frac_set_frame_async(ctx_, plane, w, h, stride));
        w_ = w;
        h_ = h;
    }
    void setFrameDeviceAsync(const void* d_plane, uint32_t w, uint32_t h, uint32_t stride)
    {
        check(frac_set_frame_device_async(ctx_, d_plane, w, h, stride));
        w_ = w;
        h_ = h;
    }
    // an external hipStream_t (as void*; nullptr: the context's own), ordered after the previous stream's work
    void setStream(void* hip_stream) { check(frac_set_stream(ctx_, hip_stream)); }
    void* stream() const { return frac_get_stream(ctx_); }
    // ABI 8: every later run writes its 32-byte tuples into dst (device memory or pinned host memory); nullptr
    // clears it
    void setTupleSink(void* dst) { check(frac_set_tuple_sink(ctx_, dst)); }
    // the last run's tuples (north_star's (domain, transform, s, o, rms)), synchronously
    void fetchTuples(frac_tuple* out) { check(frac_fetch_tuples(ctx_, out)); }
    // per-run device times since the previous call (FRAC_FLAG_TIMING, Params::timing)
    std::vector<frac_run_timing> timingHistory()
    {
        size_t n = 0;
        check(frac_timing_history(ctx_, nullptr, 0, &n));
        std::vector<frac_run_timing> out(n);
        check(frac_timing_history(ctx_, out.data(), out.size(), &n));
        out.resize(n);
        return out;
    }
    void setDomains(const std::vector<frac_grid_item>& d) { check(frac_set_domains(ctx_, d.data(), d.size())); }
    void setRanges(const frac_grid_item* r, size_t n) { check(frac_set_ranges(ctx_, r, n)); }
    void run() { check(frac_run(ctx_)); }
    void sync() { check(frac_sync(ctx_)); }
    void fetch(frac_encode_item* out, frac_stats* st = nullptr)
    {
        frac_stats tmp{};
        check(frac_fetch(ctx_, out, st ? st : &tmp));
    }
    std::vector<frac_encode_item> search(const std::vector<frac_grid_item>& ranges, frac_stats* st = nullptr)
    {
        std::vector<frac_encode_item> out(ranges.size());
        frac_stats tmp{};
        check(frac_search(ctx_, ranges.data(), ranges.size(), out.data(), st ? st : &tmp));
        return out;
    }
    std::vector<frac_grid_item> classify(std::vector<frac_grid_item> items)
    {
        check(frac_classify_items(ctx_, items.data(), items.size(), 0));
        return items;
    }
    std::vector<frac_encode_item> encodeQuadtree(uint32_t max_size, uint32_t min_size, double split_distance,
                                                 frac_stats* st = nullptr)
    {
        const frac_quadtree_params qp{max_size, min_size, split_distance};
        size_t cap = (size_t)(w_ / min_size) * (h_ / min_size), n = 0;
        std::vector<frac_encode_item> out(cap);
        frac_stats tmp{};
        check(frac_encode_quadtree(ctx_, &qp, out.data(), cap, &n, st ? st : &tmp));
        out.resize(n);
        return out;
    }
    // the same partition as 32-byte frac_qt_leaf items (ABI 7): half the bytes of encodeQuadtree's records
    std::vector<frac_qt_leaf> encodeQuadtreeLeaves(uint32_t max_size, uint32_t min_size, double split_distance,
                                                   frac_stats* st = nullptr)
    {
        const frac_quadtree_params qp{max_size, min_size, split_distance};
        size_t cap = (size_t)(w_ / min_size) * (h_ / min_size), n = 0;
        std::vector<frac_qt_leaf> out(cap);
        frac_stats tmp{};
        check(frac_encode_quadtree_leaves(ctx_, &qp, out.data(), cap, &n, st ? st : &tmp));
        out.resize(n);
        return out;
    }
    // Decoder2::decode (encode/Encoder2.hpp:67-88); plane holds the caller's initial target
    // (main.cpp zeroes it) and receives the result.  Returns {iterations, rms}.
    std::pair<int, double> decode(const std::vector<frac_encode_item>& items, uint32_t w, uint32_t h,
                                  std::vector<uint8_t>& plane, int max_iter = -1, double rms_eps = 1e-5)
    {
        plane.resize((size_t)w * h);
        int it = 0;
        double rms = 0.0;
        check(frac_decode(ctx_, items.data(), items.size(), w, h, max_iter, rms_eps, plane.data(), &it, &rms));
        return {it, rms};
    }

private:
    void check(int rc) const
    {
        if (rc != FRAC_OK)
            throw Error(std::string("fracenc: ") + frac_last_error(ctx_));
    }
    frac_ctx* ctx_ = nullptr;
    uint32_t w_ = 0, h_ = 0;
};

// EncodingEngineCore2's role with batch claims.  One engine per entry of `devices` (a device
// may repeat: several contexts and streams on one GPU), each on its own host thread; the frame
// and domain grid are set once per engine, then every engine claims `batch` ranges at a time.
class EncodingEngineCore {
public:
    EncodingEngineCore(const Params& p, std::vector<int> devices, size_t batch = 65536)
        : params_(p), batch_(batch ? batch : 1)
    {
        if (devices.empty())
            devices.push_back(0);
        for (int d : devices)
            engines_.emplace_back(d, p);
    }

    size_t engineCount() const { return engines_.size(); }

    std::vector<frac_encode_item> encode(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride,
                                         const std::vector<frac_grid_item>& domains,
                                         const std::vector<frac_grid_item>& ranges, frac_stats* total = nullptr)
    {
        std::vector<frac_encode_item> out(ranges.size());
        std::atomic<size_t> next{0};
        std::mutex m;
        frac_stats sum{};
        std::string err;
        auto worker = [&](Engine& e) {
            try {
                e.setFrame(plane, w, h, stride);
                e.setDomains(domains);
                for (;;) {
                    const size_t b0 = next.fetch_add(batch_);
                    if (b0 >= ranges.size())
                        break;
                    const size_t nb = std::min(batch_, ranges.size() - b0);
                    e.setRanges(ranges.data() + b0, nb);
                    e.run();
                    frac_stats st{};
                    e.fetch(out.data() + b0, &st);
                    std::lock_guard<std::mutex> lk(m);
                    sum.rejected_mappings += st.rejected_mappings;
                    sum.total_mappings += st.total_mappings;
                    sum.hit_ranges += st.hit_ranges;
                    sum.fallback_ranges += st.fallback_ranges;
                    sum.empty_ranges += st.empty_ranges;
                    sum.engine = st.engine;
                    sum.search_form = st.search_form;
                    sum.matrix_flops += st.matrix_flops;
                    sum.evaluated_mappings += st.evaluated_mappings;
                }
            } catch (const std::exception& ex) {
                std::lock_guard<std::mutex> lk(m);
                err = ex.what();
                next.store(ranges.size()); // stop the other engines' claims
            }
        };
        std::vector<std::thread> pool;
        for (auto& e : engines_)
            pool.emplace_back(worker, std::ref(e));
        for (auto& t : pool)
            t.join();
        if (!err.empty())
            throw Error(err);
        if (total)
            *total = sum;
        return out;
    }

private:
    Params params_;
    size_t batch_;
    std::vector<Engine> engines_;
};

// Frac::Quantizer<T> (encode/Quantizer.hpp:7-45).  value() is computed as the FMA-built
// reference does: fl(fma(q, step, min) + step/2) (GCC contracts q·step + min).
template <typename T>
class Quantizer {
public:
    using Int = uint64_t;
    Quantizer(T minValue, T maxValue, int numberOfBits)
        : min_(minValue), max_(maxValue), bits_(numberOfBits),
          step_(std::abs(maxValue - minValue) / (T)((Int)1 << numberOfBits)),
          maxQuantized_(((Int)1 << numberOfBits) - 1)
    {
        if (!(maxValue > minValue) || numberOfBits <= 1 || numberOfBits > 63)
            throw Error("Quantizer: needs max > min and 1 < bits < 64 (Quantizer.hpp:19-22)");
    }
    Int quantized(T value) const
    {
        const T q = std::floor((value - min_) / step_);
        return std::min(maxQuantized_, (Int)q);
    }
    T value(Int quant) const { return std::fma((T)quant, step_, min_) + step_ / 2; }
    T step() const { return step_; }

private:
    T min_, max_;
    int bits_;
    T step_;
    Int maxQuantized_;
};

} // namespace fracenc

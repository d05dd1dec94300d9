// HipEncodingEngine2.hpp — the reference-side binding of the MI355X engine (include/fracenc.h).
//
// A Frac2::AbstractEncodingEngine2 (sebsgit/fractencode encode/EncodingEngine2.hpp:50-85) that a
// maintainer registers in EncodingEngineCore2's engine slot (encode/EncodingEngine2.cpp:21-29, the
// commented OpenCL block):
//
//     try {
//         auto engine = std::make_unique<Frac2::HipEncodingEngine2>(params, image, gridSource);
//         engine->setName("HIP");
//         this->_engines.push_back(std::move(engine));
//     } catch (const std::exception& exc) { std::cout << "failed to create engine: " << exc.what(); }
//
// It uses only the base class's public and protected interface — no change to the reference's
// classes:
//   * the constructor uploads the plane and the domain grid; the library validates the grid there
//     (one item size, inside the plane, categories −1..5), so an unusable grid throws where
//     EncodingEngine2.cpp:27-29 catches and logs "failed to create engine";
//   * encode(item) (virtual, EncodingEngine2.hpp:63-66) only records the claimed item;
//   * finalize() (run by the core on the engine's thread once the queue is empty,
//     EncodingEngine2.hpp:144-145) searches every claimed item in ONE frac_search on the GPU,
//     then hands each item to the base AbstractEncodingEngine2::encode, whose encode_impl call
//     returns the precomputed record — so the base class's private result list and task counter
//     fill exactly as for a CPU engine.  finalize() never lets an exception out: it runs on the
//     core's worker thread with no handler (EncodingEngine2.hpp:144-145), where a throw would be
//     std::terminate.  A failure (a HIP error, a range geometry the engine refuses) is kept, the
//     claimed items produce no records, and rethrowIfFailed() rethrows it on the caller's thread
//     after EncodingEngineCore2::encode returns (Encoder2.hpp:38) — see INTEGRATION.md.
// The reference claims one range per mutex round trip (EncodingEngine2.hpp:131-140): batching it
// on the device side is what makes a GPU engine pay off (the dormant OpenCL engine launched a
// blocking kernel per item, gpu/opencl/OpenCLEncodingEngine.cpp:294-330).
//
// Compiled against the reference headers by tests/test_integration.py (static_asserts below) and
// run through the reference's own EncodingEngineCore2 by oracle/ref/core_driver.cpp.
#pragma once

#include "encode/EncodingEngine2.hpp"
#include "fracenc.h"

#include <chrono>
#include <cstddef>
#include <exception>
#include <stdexcept>
#include <string>
#include <vector>

namespace Frac2 {

// the C ABI's records are the reference's, byte for byte (encode/datatypes.h:8-26,
// image/partition2.hpp:93-99): the binding passes the reference's arrays straight through
static_assert(sizeof(frac_grid_item) == sizeof(UniformGridItem), "UniformGridItem layout");
static_assert(offsetof(GridItemBase, origin) == offsetof(frac_grid_item, x), "GridItemBase origin");
static_assert(offsetof(GridItemBase, size) == offsetof(frac_grid_item, w), "GridItemBase size");
static_assert(sizeof(frac_score) == sizeof(Frac::transform_score_t), "transform_score_t layout");
static_assert(offsetof(Frac::transform_score_t, distance) == offsetof(frac_score, distance), "distance");
static_assert(offsetof(Frac::transform_score_t, contrast) == offsetof(frac_score, contrast), "contrast");
static_assert(offsetof(Frac::transform_score_t, brightness) == offsetof(frac_score, brightness), "brightness");
static_assert(offsetof(Frac::transform_score_t, transform) == offsetof(frac_score, transform), "transform");
static_assert(sizeof(frac_match) == sizeof(Frac::item_match_t), "item_match_t layout");
static_assert(offsetof(Frac::item_match_t, x) == offsetof(frac_match, x), "item_match_t x");
static_assert(offsetof(Frac::item_match_t, sourceItemSize) == offsetof(frac_match, sw), "item_match_t size");
static_assert(sizeof(frac_encode_item) == sizeof(Frac::encode_item_t), "encode_item_t layout");
static_assert(offsetof(Frac::encode_item_t, match) == offsetof(frac_encode_item, match), "encode_item_t match");
static_assert(sizeof(Frac::TransformType) == sizeof(int32_t), "TransformType is an int");

class HipEncodingEngine2 : public AbstractEncodingEngine2 {
public:
    // transforms: 4 = TransformMatcher::match (transformmatcher.h:41-45); the classifier follows the
    // CLI's --noclassifier (main.cpp:152-153); `engine` one of FRAC_ENGINE_*
    HipEncodingEngine2(const encode_parameters_t& params, const ImagePlane& sourceImage, const UniformGrid& sourceGrid,
                       int device = 0, uint32_t engine = FRAC_ENGINE_AUTO)
        : AbstractEncodingEngine2(params, sourceImage, sourceGrid)
    {
        frac_params fp{};
        fp.transforms = 4;
        fp.use_classifier = params.noclassifier ? 0 : 1;
        fp.rms_threshold = params.rmsThreshold;
        fp.s_max = params.sMax;
        fp.engine = engine;
        fp.flags = 0;
        _ctx = frac_create(device, &fp);
        if (!_ctx)
            throw std::runtime_error(std::string("frac_create: ") + frac_last_error(nullptr));
        const auto& doms = sourceGrid.items(); // categories as preclassified at grid build (main.cpp:155-161)
        try {
            check(frac_set_frame(_ctx, sourceImage.data(), sourceImage.width(), sourceImage.height(),
                                 sourceImage.stride()));
            check(frac_set_domains(_ctx, reinterpret_cast<const frac_grid_item*>(doms.data()), doms.size()));
        } catch (...) {
            frac_destroy(_ctx);
            throw;
        }
    }
    ~HipEncodingEngine2() override { frac_destroy(_ctx); }
    HipEncodingEngine2(const HipEncodingEngine2&) = delete;
    HipEncodingEngine2& operator=(const HipEncodingEngine2&) = delete;

    // a claim: recorded, searched in finalize()
    void encode(const UniformGridItem& targetItem) override { _pending.push_back(targetItem); }

    // one batched search over every claimed range, then the base class records the results; on
    // the core's worker thread, so nothing may escape (see the header comment)
    void finalize() noexcept override
    {
        try {
            using Clock = std::chrono::steady_clock;
            const auto t0 = Clock::now();
            _records.resize(_pending.size());
            frac_stats st{};
            // frac_search's three steps, timed apart (the drop-in measurement's breakdown)
            check(frac_set_ranges(_ctx, reinterpret_cast<const frac_grid_item*>(_pending.data()), _pending.size()));
            check(frac_run(_ctx)); // preparation for these ranges (host), then every launch (asynchronous)
            const auto tr = Clock::now();
            check(frac_sync(_ctx));
            const auto ts = Clock::now();
            check(frac_fetch(_ctx, reinterpret_cast<frac_encode_item*>(_records.data()), &st));
            const auto t1 = Clock::now();
            _prepareSeconds += std::chrono::duration<double>(tr - t0).count();
            _deviceSeconds += std::chrono::duration<double>(ts - tr).count();
            _fetchSeconds += std::chrono::duration<double>(t1 - ts).count();
            _rejected += st.rejected_mappings;
            _next = 0;
            for (const auto& item : _pending)
                AbstractEncodingEngine2::encode(item); // → encode_impl → _records[_next++]
            _searched += _pending.size();
            _searchSeconds += std::chrono::duration<double>(t1 - t0).count();
            _handbackSeconds += std::chrono::duration<double>(Clock::now() - t1).count();
        } catch (...) {
            _failed = std::current_exception();
            _lost += _pending.size();
        }
        _pending.clear();
        _records.clear();
    }

    // On the caller's thread after EncodingEngineCore2::encode: rethrows a failure of finalize()
    // (whose claimed ranges then have no record in the core's result).
    void rethrowIfFailed() const
    {
        if (_failed)
            std::rethrow_exception(_failed);
    }
    bool failed() const noexcept { return _failed != nullptr; }

    // TransformEstimator2::rejectedMappings() of the ranges this engine searched
    uint64_t rejectedMappings() const noexcept { return _rejected; }
    // ranges searched by this engine / claimed but lost to a failure
    size_t searchedRanges() const noexcept { return _searched; }
    size_t lostRanges() const noexcept { return _lost; }
    // seconds finalize() spent in frac_search (upload of the claims, search, records back) and handing the
    // records to the base class's encode() (the core's per-item result list)
    double searchSeconds() const noexcept { return _searchSeconds; }
    double handbackSeconds() const noexcept { return _handbackSeconds; }
    // the search's parts: claims up + preparation + launches (host), the device work after them, the records
    // and statistics back
    double prepareSeconds() const noexcept { return _prepareSeconds; }
    double deviceSeconds() const noexcept { return _deviceSeconds; }
    double fetchSeconds() const noexcept { return _fetchSeconds; }

protected:
    encode_item_t encode_impl(const UniformGridItem& targetItem) const override
    {
        if (_next >= _records.size())
            throw std::logic_error("HipEncodingEngine2: encode_impl outside finalize()");
        const encode_item_t& e = _records[_next++];
        if (e.x != targetItem.origin.x() || e.y != targetItem.origin.y())
            throw std::logic_error("HipEncodingEngine2: record order");
        return e;
    }

private:
    void check(int rc) const
    {
        if (rc != FRAC_OK)
            throw std::runtime_error(std::string("fracenc: ") + frac_last_error(_ctx));
    }
    frac_ctx* _ctx = nullptr;
    std::vector<UniformGridItem> _pending;
    std::vector<encode_item_t> _records;
    mutable size_t _next = 0;
    uint64_t _rejected = 0;
    size_t _searched = 0, _lost = 0;
    double _searchSeconds = 0.0, _handbackSeconds = 0.0, _prepareSeconds = 0.0, _deviceSeconds = 0.0,
           _fetchSeconds = 0.0;
    std::exception_ptr _failed;
};

} // namespace Frac2

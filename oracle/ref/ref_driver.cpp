// ref_driver.cpp — thin C-ABI driver around the UNMODIFIED reference sources.
//
// TEST INFRASTRUCTURE ONLY.  This file is ours; everything it calls lives under
// /root/reference and is compiled from there by oracle/ref/Makefile into
// oracle/_ref/libfracref.so (git-ignored, travels to the GPU box as a built .so).
// Only tests/, bench.py's cpu_baseline leg and tools/make_golden.py load it.
//
// What it drives (reference file:line):
//   grid construction      image/partition2.hpp:109-135 via main.cpp:142-162 (encode_image2)
//   classifier pre-pass    encode/Classifier2.cpp:64-68 (preclassify on the SOURCE plane for both grids)
//   T=4 search             encode/TransformEstimator2.hpp:29-48 (TransformEstimator2::estimate)
//   T=8 search ("driver B") the same loop as estimate() but calling the reference's public
//                          TransformMatcher::matchTransformTypes<8 types> (encode/transformmatcher.h:59-68)
//   decode                 encode/Encoder2.hpp:67-99 (Decoder2)
//   colour load            image/ImageIO.cpp:60-66 (stb load + rgb2yuv)
//
// Threading: EncodingEngineCore2 hard-codes hardware_concurrency() workers
// (encode/EncodingEngine2.cpp:12-20).  To time the reference on a stated core
// count we run TransformEstimator2::estimate (the hot path itself) from our own
// worker pool with the same one-range-per-claim queue discipline.
#include "encode/TransformEstimator2.hpp"
#include "encode/Classifier2.hpp"
#include "encode/Encoder2.hpp"
#include "encode/transformmatcher.h"
#include "encode/Quantizer.hpp"
#include "image/ImageIO.hpp"
#include "image/partition2.hpp"

#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

using namespace Frac2;
using Frac::TransformType;

extern "C" {

struct fr_result {
    uint32_t x, y;      // range origin
    uint32_t dx, dy;    // winning domain origin
    uint32_t dw, dh;    // winning domain size (0,0 when no candidate)
    int32_t transform;
    int32_t pad;
    double distance, contrast, brightness;
};

static ImagePlane make_plane(const uint8_t* p, uint32_t w, uint32_t h, uint32_t stride)
{
    std::vector<uint8_t> buf(p, p + size_t(h) * stride);
    return ImagePlane(Size32u(w, h), stride, std::move(buf));
}

int fr_load_yuv(const char* path, uint8_t* y, uint8_t* u, uint8_t* v, uint32_t* w, uint32_t* h)
{
    auto planes = ImageIO::loadImage(path);
    const uint32_t W = planes[0].width(), H = planes[0].height();
    if (w) *w = W;
    if (h) *h = H;
    if (y)
        for (uint32_t r = 0; r < H; ++r)
            std::memcpy(y + size_t(r) * W, planes[0].data() + size_t(r) * planes[0].stride(), W);
    for (int c = 1; c < 3; ++c) {
        uint8_t* dst = c == 1 ? u : v;
        if (!dst)
            continue;
        const uint32_t cw = planes[c].width(), ch = planes[c].height();
        for (uint32_t r = 0; r < ch; ++r)
            std::memcpy(dst + size_t(r) * cw, planes[c].data() + size_t(r) * planes[c].stride(), cw);
    }
    return 0;
}

int fr_category(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride, uint32_t x, uint32_t y, uint32_t size)
{
    auto img = make_plane(plane, w, h, stride);
    UniformGridItem it(Point2du(x, y), Size32u(size, size));
    return BrightnessBlocksClassifier2::getCategory(img, it);
}

// Builds the domain/range grids exactly as main.cpp:142-162 does and runs the
// reference search for the selected ranges (all ranges when sel == nullptr).
// out[] is indexed like sel (or like the range grid when sel == nullptr).
int fr_estimate(const uint8_t* src, const uint8_t* tgt, uint32_t w, uint32_t h, uint32_t stride,
                uint32_t src_size, uint32_t tgt_size, int ntransforms, double thr, double smax,
                int use_classifier, int nthreads, const uint32_t* sel, size_t nsel,
                fr_result* out, uint64_t* rejected, double time_budget_s, size_t* n_done)
{
    auto srcImg = make_plane(src, w, h, stride);
    auto tgtImg = make_plane(tgt, w, h, stride);
    std::unique_ptr<Classifier2> classifier;
    if (use_classifier)
        classifier = std::make_unique<BrightnessBlocksClassifier2>(srcImg, tgtImg);
    else
        classifier = std::make_unique<DummyClassifier>(srcImg, tgtImg);
    const Classifier2* cls = classifier.get();
    auto cb = [&](const Point2du& origin, const Size32u& size) {
        UniformGridItem::ExtraData data;
        cls->preclassify(origin, size, data);
        return data;
    };
    const Size32u srcSz(src_size, src_size), tgtSz(tgt_size, tgt_size);
    const Size32u off = srcSz / 2; // latticeSize = 2 (encode/encode_parameters.h:8)
    auto sourceGrid = createUniformGrid(Size32u(w, h), srcSz, off, cb);
    auto targetGrid = createUniformGrid(Size32u(w, h), tgtSz, tgtSz, cb);
    auto matcher = std::make_shared<TransformMatcher>(thr, smax);
    TransformEstimator2 estimator(srcImg, tgtImg, std::move(classifier), matcher, sourceGrid);
    const auto& ranges = targetGrid.items();
    const size_t count = sel ? nsel : ranges.size();
    std::atomic<size_t> next{0};
    std::atomic<uint64_t> rej8{0};
    std::atomic<size_t> done{0};
    const auto t0 = std::chrono::steady_clock::now();

    auto run8 = [&](const UniformGridItem& r) {
        // Driver B: estimate()'s loop verbatim, with the 8-transform chain.
        item_match_t result;
        for (const auto& d : sourceGrid.items()) {
            if (cls->compare(d, r)) {
                auto score = matcher->matchTransformTypes<TransformType::Id, TransformType::Rotate_90,
                    TransformType::Rotate_180, TransformType::Rotate_270, TransformType::Flip,
                    TransformType::Flip_Rotate_90, TransformType::Flip_Rotate_180,
                    TransformType::Flip_Rotate_270>(srcImg, d, tgtImg, r, transform_score_t{});
                if (score.distance < result.score.distance) {
                    result.score = score;
                    result.x = d.origin.x();
                    result.y = d.origin.y();
                    result.sourceItemSize = d.size;
                }
                if (matcher->checkDistance(result.score.distance))
                    break;
            } else {
                ++rej8;
            }
        }
        return result;
    };
    auto worker = [&]() {
        while (true) {
            if (time_budget_s > 0.0) {
                std::chrono::duration<double> el = std::chrono::steady_clock::now() - t0;
                if (el.count() > time_budget_s)
                    return;
            }
            const size_t i = next.fetch_add(1);
            if (i >= count)
                return;
            const auto& r = ranges.at(sel ? sel[i] : i);
            item_match_t m = ntransforms == 8 ? run8(r) : estimator.estimate(r);
            fr_result& o = out[i];
            o.x = r.origin.x();
            o.y = r.origin.y();
            o.dx = m.x;
            o.dy = m.y;
            o.dw = m.sourceItemSize.x();
            o.dh = m.sourceItemSize.y();
            o.transform = static_cast<int32_t>(m.score.transform);
            o.pad = 0;
            o.distance = m.score.distance;
            o.contrast = m.score.contrast;
            o.brightness = m.score.brightness;
            ++done;
        }
    };
    const int nt = nthreads > 0 ? nthreads : 1;
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t)
        pool.emplace_back(worker);
    for (auto& t : pool)
        t.join();
    if (rejected)
        *rejected = ntransforms == 8 ? rej8.load() : estimator.rejectedMappings();
    if (n_done)
        *n_done = done.load();
    return 0;
}

// createUniformGrid (image/partition2.hpp:109-135) with the reference's Size32u item size and
// offset (tests/OpenCLTest.cpp:76-78 uses 4×4 items at offset (4, 2)).  Returns the item count,
// writes at most cap items {x, y, w, h, category = -1}.
struct fr_item {
    uint32_t x, y, w, h;
    int32_t category;
};

size_t fr_uniform_grid(uint32_t w, uint32_t h, uint32_t sw, uint32_t sh, uint32_t ox, uint32_t oy, fr_item* out,
                       size_t cap)
{
    const auto grid = createUniformGrid(Size32u(w, h), Size32u(sw, sh), Size32u(ox, oy));
    const auto& items = grid.items();
    for (size_t i = 0; i < items.size() && i < cap; ++i)
        out[i] = fr_item{items[i].origin.x(), items[i].origin.y(), items[i].size.x(), items[i].size.y(),
                         items[i].data.bb_classifierBin};
    return items.size();
}

// BrightnessBlocksClassifier2::preclassify (encode/Classifier2.cpp:64-68) of arbitrary items on
// `plane` (the grid-build callback of main.cpp:155-159 and tests/OpenCLTest.cpp:79-84).
int fr_classify_items(const uint8_t* plane, uint32_t w, uint32_t h, uint32_t stride, fr_item* items, size_t n)
{
    auto img = make_plane(plane, w, h, stride);
    BrightnessBlocksClassifier2 classifier(img, img);
    for (size_t i = 0; i < n; ++i) {
        UniformGridItem::ExtraData data;
        classifier.preclassify(Point2du(items[i].x, items[i].y), Size32u(items[i].w, items[i].h), data);
        items[i].category = data.bb_classifierBin;
    }
    return 0;
}

// TransformEstimator2::estimate (encode/TransformEstimator2.hpp:29-48) over caller-given domain and
// range item lists — any item sizes the reference's types hold (Size32u: rectangles included) —
// with the classifier categories preclassified on the source plane as main.cpp:155-161 does.
// out[] and the reject count as fr_estimate; single-threaded.
int fr_estimate_items(const uint8_t* src, const uint8_t* tgt, uint32_t w, uint32_t h, uint32_t stride,
                      const fr_item* doms, size_t nd, const fr_item* rngs, size_t nr, int ntransforms, double thr,
                      double smax, int use_classifier, fr_result* out, uint64_t* rejected)
{
    auto srcImg = make_plane(src, w, h, stride);
    auto tgtImg = make_plane(tgt, w, h, stride);
    std::unique_ptr<Classifier2> classifier;
    if (use_classifier)
        classifier = std::make_unique<BrightnessBlocksClassifier2>(srcImg, tgtImg);
    else
        classifier = std::make_unique<DummyClassifier>(srcImg, tgtImg);
    UniformGrid sourceGrid = UniformGrid::createEmpty(0);
    std::vector<UniformGridItem> ranges;
    for (size_t i = 0; i < nd; ++i) {
        UniformGridItem::ExtraData data;
        classifier->preclassify(Point2du(doms[i].x, doms[i].y), Size32u(doms[i].w, doms[i].h), data);
        sourceGrid.add(Point2du(doms[i].x, doms[i].y), Size32u(doms[i].w, doms[i].h), std::move(data));
    }
    for (size_t i = 0; i < nr; ++i) {
        UniformGridItem::ExtraData data;
        classifier->preclassify(Point2du(rngs[i].x, rngs[i].y), Size32u(rngs[i].w, rngs[i].h), data);
        ranges.push_back(UniformGridItem(Point2du(rngs[i].x, rngs[i].y), Size32u(rngs[i].w, rngs[i].h), std::move(data)));
    }
    auto matcher = std::make_shared<TransformMatcher>(thr, smax);
    const Classifier2* cls = classifier.get();
    TransformEstimator2 estimator(srcImg, tgtImg, std::move(classifier), matcher, sourceGrid);
    uint64_t rej8 = 0;
    auto run8 = [&](const UniformGridItem& r) { // driver B (fr_estimate): estimate()'s loop, 8-transform chain
        item_match_t result;
        for (const auto& d : sourceGrid.items()) {
            if (cls->compare(d, r)) {
                auto score = matcher->matchTransformTypes<TransformType::Id, TransformType::Rotate_90,
                    TransformType::Rotate_180, TransformType::Rotate_270, TransformType::Flip,
                    TransformType::Flip_Rotate_90, TransformType::Flip_Rotate_180,
                    TransformType::Flip_Rotate_270>(srcImg, d, tgtImg, r, transform_score_t{});
                if (score.distance < result.score.distance) {
                    result.score = score;
                    result.x = d.origin.x();
                    result.y = d.origin.y();
                    result.sourceItemSize = d.size;
                }
                if (matcher->checkDistance(result.score.distance))
                    break;
            } else {
                ++rej8;
            }
        }
        return result;
    };
    for (size_t i = 0; i < nr; ++i) {
        const item_match_t m = ntransforms == 8 ? run8(ranges[i]) : estimator.estimate(ranges[i]);
        fr_result& o = out[i];
        o.x = ranges[i].origin.x();
        o.y = ranges[i].origin.y();
        o.dx = m.x;
        o.dy = m.y;
        o.dw = m.sourceItemSize.x();
        o.dh = m.sourceItemSize.y();
        o.transform = static_cast<int32_t>(m.score.transform);
        o.pad = 0;
        o.distance = m.score.distance;
        o.contrast = m.score.contrast;
        o.brightness = m.score.brightness;
    }
    if (rejected)
        *rejected = ntransforms == 8 ? rej8 : estimator.rejectedMappings();
    return 0;
}

// Full reference decode (encode/Encoder2.hpp:67-99) of an encoding given as
// fr_result records in range order; returns iterations, writes the plane.
int fr_decode(const fr_result* recs, size_t n, uint32_t tgt_size, uint32_t w, uint32_t h,
              int max_iter, double rms_eps, uint8_t* out_plane, double* out_rms)
{
    grid_encode_data_t data;
    for (size_t i = 0; i < n; ++i) {
        encode_item_t e;
        e.x = recs[i].x;
        e.y = recs[i].y;
        e.w = tgt_size;
        e.h = tgt_size;
        e.match.x = recs[i].dx;
        e.match.y = recs[i].dy;
        e.match.sourceItemSize = Size32u(recs[i].dw, recs[i].dh);
        e.match.score.distance = recs[i].distance;
        e.match.score.contrast = recs[i].contrast;
        e.match.score.brightness = recs[i].brightness;
        e.match.score.transform = static_cast<TransformType>(recs[i].transform);
        data.encoded.push_back(e);
    }
    std::vector<uint8_t> buf(size_t(w) * h, 0);
    ImagePlane result(Size32u(w, h), w, std::move(buf));
    Decoder2 decoder(result, max_iter, rms_eps, false);
    auto stats = decoder.decode(data);
    for (uint32_t r = 0; r < h; ++r)
        std::memcpy(out_plane + size_t(r) * w, result.data() + size_t(r) * result.stride(), w);
    if (out_rms)
        *out_rms = stats.rms;
    return stats.iterations;
}

// ImageIO::rgb2yuv (image/ImageIO.cpp:43-58) on a caller-supplied packed RGB buffer.
int fr_rgb2yuv(const uint8_t* rgb, uint32_t w, uint32_t h, uint32_t rgb_stride, uint8_t* y, uint32_t ys, uint8_t* u,
               uint32_t us, uint8_t* v, uint32_t vs)
{
    const std::ptrdiff_t uvh = (h + 1) / 2;
    ImageIO::rgb2yuv({rgb, static_cast<std::ptrdiff_t>(size_t(rgb_stride) * h)}, w, h, rgb_stride,
                     {y, static_cast<std::ptrdiff_t>(size_t(ys) * h)}, ys,
                     {u, static_cast<std::ptrdiff_t>(size_t(us) * uvh)}, us,
                     {v, static_cast<std::ptrdiff_t>(size_t(vs) * uvh)}, vs);
    return 0;
}

// Frac::Quantizer<double> (encode/Quantizer.hpp:7-45): quantized() and value() of n values.
int fr_quantize(double vmin, double vmax, int bits, const double* v, size_t n, uint64_t* q, double* back)
{
    Frac::Quantizerd qz(vmin, vmax, bits);
    for (size_t i = 0; i < n; ++i) {
        q[i] = qz.quantized(v[i]);
        back[i] = qz.value(q[i]);
    }
    return 0;
}

} // extern "C"

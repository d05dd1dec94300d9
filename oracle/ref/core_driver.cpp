// core_driver.cpp — runs the REFERENCE's EncodingEngineCore2 (encode/EncodingEngine2.hpp:115-180,
// EncodingEngine2.cpp:7-30, compiled unmodified from /root/reference) with the HIP engine of
// integration/HipEncodingEngine2.hpp registered — alone (--nocpu, main.cpp:83-84), or beside the
// reference's hardware_concurrency CPU engines sharing the one claim queue (the default CLI).
//
// TEST INFRASTRUCTURE (tests/test_integration.py).  The reference registers accelerator engines
// inside EncodingEngineCore2's constructor (EncodingEngine2.cpp:21-29, the commented OpenCL block);
// a maintainer adds the three lines there.  This driver cannot edit the reference, so it performs
// the same push_back into the core's private engine list through the standard explicit-
// instantiation access idiom (access checks do not apply to explicit instantiations,
// [temp.spec.general]/6) — the registration itself, nothing else.
//
// usage: core_driver PLANE.u8 W H SRC TGT CLASSIFIER(0|1) RMS_THR SMAX OUT.bin [CPU [DEVICES]]
//   CPU: 0 = --nocpu (main.cpp:83-84); k > 0 = k of the reference's CpuEncodingEngine2 on the queue, registered
//   here (the core's constructor would make hardware_concurrency() of them — 256 on the GPU box against a
//   16-CPU quota — and EncodingEngineCore2::encode's completion wait can lose its last wakeup when that many
//   engines finish together: it re-waits on the condition variable without a predicate after a yield,
//   EncodingEngine2.hpp:154-160.  A watchdog turns such a hang into exit 7 instead of a silent stall).
//   DEVICES: a comma list of HIP devices, one HipEncodingEngine2 registered per entry (default "0";
//   "0,0" = two engines, two contexts, on device 0 — the one-GPU box's stand-in for one engine per
//   device; "all" = one per device frac_device_count() reports).
//   MODE (optional): "ref" (default) = the reference's EncodingEngineCore2::encode; "batch:K" = the maintainer
//   patch INTEGRATION.md §Drop-in rate proposes, restated here over the same engines (one lock claims up to K
//   items, no yield per item, a predicate wait) — for timing the patch, never for parity.
//   A tail engine (below) is registered last in "ref" mode: the core's lost final wakeup cannot happen.
//   stdout: one JSON line {"encode_s", "records_s", "tail_hold_s", "drop_in_s", "construct_s", ...} —
//   core.encode()'s wall time, the time the last real engine's finalize() returned, the tail's hold,
//   encode_s − tail_hold_s (the core's time with a wait that loses nothing), and the construction of the core
//   and its engines before it (HIP runtime start, frame and domain upload: inside Encoder2's timer too).
//   OUT.bin: the core's result().encoded (encode_item_t, 64 B each) in the core's order, then the
//   rejected-mapping count of the whole search (u64: the CPU engines' estimator plus the HIP
//   engines'), the number of ranges the HIP engines searched (u64), each HIP engine's own count
//   (u64 each, in registration order) and the number of HIP engines (u64).
//   Exit 6 (message on stderr) when a HIP engine's finalize() failed: rethrowIfFailed() on this
//   thread, after the core's workers have joined — not std::terminate on a worker.
#include "encode/EncodingEngine2.hpp"
#include "encode/Classifier2.hpp"
#include "encode/TransformEstimator2.hpp"
#include "image/partition2.hpp"
#include "HipEncodingEngine2.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unistd.h>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

using namespace Frac2;

namespace {
using Engines = std::vector<std::unique_ptr<AbstractEncodingEngine2>>;
template <Engines EncodingEngineCore2::*M>
struct EnginesOf {
    friend Engines& engines_of(EncodingEngineCore2& c) { return c.*M; }
};
Engines& engines_of(EncodingEngineCore2& c);
template struct EnginesOf<&EncodingEngineCore2::_engines>;

struct NullReporter : ProgressReporter2 {
    void log(size_t, size_t) override {}
};

using Clock = std::chrono::steady_clock;

// counts the registered engines whose finalize() has returned (the tail engine waits for all of them)
struct FinishLine {
    std::mutex m;
    std::condition_variable cv;
    size_t done = 0;
    Clock::time_point last{};
    void arrive()
    {
        std::lock_guard<std::mutex> lock(m);
        ++done;
        last = Clock::now();
        cv.notify_all();
    }
};

// an engine of the core that reports its finalize() to the finish line (no other change)
template <class E>
class Counted : public E {
public:
    template <class... A>
    Counted(FinishLine& line, A&&... a) : E(std::forward<A>(a)...), _line(line) {}
    void finalize() noexcept override
    {
        E::finalize();
        _line.arrive();
    }

private:
    FinishLine& _line;
};

// The lost-wakeup fix by construction.  EncodingEngineCore2::encode waits on queueEmpty
// without a predicate and, after each wakeup, yields before it waits again (EncodingEngine2.hpp:156-161): a
// worker's notify_one that lands in that window is lost, and when it was the last one the core never returns.
// The tail engine is registered last; its init() (run on its own worker thread before that worker claims
// anything, EncodingEngine2.hpp:128) blocks until every other engine's finalize() has returned — the queue is
// then empty, so the tail never claims a range — and `hold` longer, so the other workers' notifications have
// all been consumed and the main thread waits again.  The tail's own notify is then the only one in flight,
// and it is the last.  (A CpuEncodingEngine2 underneath: were it ever to claim a range it would encode it.)
class TailEngine : public CpuEncodingEngine2 {
public:
    TailEngine(FinishLine& line, size_t others, std::chrono::milliseconds hold, const encode_parameters_t& params,
               const ImagePlane& image, const UniformGrid& grid, const TransformEstimator2& estimator)
        : CpuEncodingEngine2(params, image, grid, estimator), _line(line), _others(others), _hold(hold)
    {
    }
    void init() override
    {
        std::unique_lock<std::mutex> lock(_line.m);
        _line.cv.wait(lock, [&] { return _line.done >= _others; });
        lock.unlock();
        std::this_thread::sleep_for(_hold);
        released = Clock::now();
    }
    Clock::time_point released{};

private:
    FinishLine& _line;
    size_t _others;
    std::chrono::milliseconds _hold;
};

// MODE batch:K — the maintainer patch of INTEGRATION.md §Drop-in rate, restated over the core's engines: the
// reference's loop (EncodingEngine2.hpp:126-168) where a HIP engine claims up to K ranges per lock (a CPU
// engine still one: it works on each for ≈0.4 s at C3), no yield per claim, and a join instead of the
// predicate-less wait.  Records are appended in engine order, as the reference's core does.
std::vector<encode_item_t> encode_batched(Engines& engines, const UniformGrid& grid, size_t K)
{
    const auto& queue = grid.items();
    std::mutex qm;
    size_t next = 0;
    std::vector<std::thread> threads;
    for (auto& e : engines) {
        AbstractEncodingEngine2* eng = e.get();
        const size_t k = dynamic_cast<HipEncodingEngine2*>(eng) ? K : 1;
        threads.emplace_back([&, eng, k] {
            eng->init();
            for (;;) {
                size_t a, b;
                {
                    std::lock_guard<std::mutex> lock(qm);
                    a = next;
                    b = std::min(queue.size(), a + k);
                    next = b;
                }
                if (a == b)
                    break;
                for (size_t i = a; i < b; ++i)
                    eng->encode(queue[i]);
            }
            eng->finalize();
        });
    }
    for (auto& t : threads)
        t.join(); // join is the predicate wait: no wakeup to lose
    std::vector<encode_item_t> out;
    for (auto& e : engines) {
        const auto part = e->result();
        out.insert(out.end(), part.begin(), part.end());
    }
    return out;
}
} // namespace

int main(int argc, char** argv)
{
    if (argc < 10 || argc > 13) {
        std::fprintf(stderr, "usage: %s PLANE W H SRC TGT CLS THR SMAX OUT [CPU [DEVICES [MODE]]]\n", argv[0]);
        return 2;
    }
    size_t batch = 0; // 0: the reference's core
    if (argc == 13 && std::strncmp(argv[12], "batch:", 6) == 0)
        batch = std::max(1, std::atoi(argv[12] + 6));
    else if (argc == 13 && std::strcmp(argv[12], "ref") != 0) {
        std::fprintf(stderr, "MODE must be ref or batch:K\n");
        return 2;
    }
    std::vector<int> devices;
    if (argc >= 12 && std::strcmp(argv[11], "all") == 0) {
        const int n = frac_device_count();
        for (int d = 0; d < n; ++d)
            devices.push_back(d);
    } else {
        std::stringstream ss(argc >= 12 ? argv[11] : "0");
        for (std::string tok; std::getline(ss, tok, ',');)
            devices.push_back(std::atoi(tok.c_str()));
    }
    if (devices.empty()) {
        std::fprintf(stderr, "no HIP device to register\n");
        return 2;
    }
    const uint32_t W = std::atoi(argv[2]), H = std::atoi(argv[3]);
    encode_parameters_t params;
    params.sourceGridSize = std::atoi(argv[4]);
    params.targetGridSize = std::atoi(argv[5]);
    params.noclassifier = std::atoi(argv[6]) == 0;
    params.rmsThreshold = std::atof(argv[7]);
    params.sMax = std::atof(argv[8]);
    const int ncpu = argc >= 11 ? std::atoi(argv[10]) : 0;
    params.nocpu = true; // the CPU engines, if any, are registered below (see the usage note)
    std::vector<uint8_t> buf(size_t(W) * H);
    {
        std::ifstream f(argv[1], std::ios::binary);
        f.read(reinterpret_cast<char*>(buf.data()), buf.size());
        if (!f)
            return 3;
    }
    ImagePlane image(Size32u(W, H), W, std::move(buf));
    // grids and classifier exactly as encode_image2 builds them (main.cpp:142-162)
    const Size32u gridSizeTarget(params.targetGridSize, params.targetGridSize);
    const Size32u gridSizeSource(params.sourceGridSize, params.sourceGridSize);
    const Size32u gridOffset = gridSizeSource / params.latticeSize;
    std::unique_ptr<Classifier2> classifier = std::make_unique<BrightnessBlocksClassifier2>(image, image);
    if (params.noclassifier)
        classifier = std::make_unique<DummyClassifier>(image, image);
    auto cb = [&](const Point2du& origin, const Size32u& size) {
        UniformGridItem::ExtraData data;
        classifier->preclassify(origin, size, data);
        return data;
    };
    auto sourceGrid = createUniformGrid(image.size(), gridSizeSource, gridOffset, cb);
    auto targetGrid = createUniformGrid(image.size(), gridSizeTarget, gridSizeTarget, cb);
    // Encoder2's estimator (encode/Encoder2.hpp:36) and core (:38)
    TransformEstimator2 estimator(image, image, std::move(classifier),
                                  std::make_shared<TransformMatcher>(params.rmsThreshold, params.sMax), sourceGrid);
    NullReporter reporter;
    // Encoder2's timer (main.cpp:164-167) starts before the core and its engines are constructed
    const auto tc = std::chrono::steady_clock::now();
    EncodingEngineCore2 core(params, image, sourceGrid, estimator, &reporter);
    FinishLine line;
    for (int i = 0; i < ncpu; ++i) { // EncodingEngine2.cpp:12-20's engines, k of them
        auto engine = std::make_unique<Counted<CpuEncodingEngine2>>(line, params, image, sourceGrid, estimator);
        engine->setName("cpu " + std::to_string(i));
        engines_of(core).push_back(std::move(engine));
    }
    uint64_t rejected = 0;
    std::vector<Counted<HipEncodingEngine2>*> hips;
    // EncodingEngine2.cpp:21-29, filled in: one engine per device; all of them
    // claim from the core's one queue (EncodingEngine2.hpp:126-168), beside the CPU engines unless --nocpu
    for (size_t i = 0; i < devices.size(); ++i) {
        try {
            auto engine = std::make_unique<Counted<HipEncodingEngine2>>(line, params, image, sourceGrid, devices[i]);
            engine->setName("HIP " + std::to_string(i));
            hips.push_back(engine.get());
            engines_of(core).push_back(std::move(engine));
        } catch (const std::exception& exc) {
            std::printf("failed to create engine: %s\n", exc.what());
            return 4;
        }
    }
    std::thread([] { // the watchdog (see the usage note): a lost wakeup in the reference's core ends the run
        std::this_thread::sleep_for(std::chrono::seconds(120));
        std::fprintf(stderr, "watchdog: EncodingEngineCore2::encode did not return in 120 s\n");
        _exit(7);
    }).detach();
    const size_t others = engines_of(core).size();
    TailEngine* tail = nullptr;
    if (!batch) {
        auto engine = std::make_unique<TailEngine>(line, others, std::chrono::milliseconds(20), params, image,
                                                   sourceGrid, estimator);
        engine->setName("tail");
        tail = engine.get();
        engines_of(core).push_back(std::move(engine));
    }
    std::vector<encode_item_t> batched;
    const auto t0 = Clock::now();
    if (batch)
        batched = encode_batched(engines_of(core), targetGrid, batch);
    else
        core.encode(targetGrid);
    const auto t1 = Clock::now();
    {
        auto sec = [&](Clock::time_point t) { return std::chrono::duration<double>(t - t0).count(); };
        const double encode_s = sec(t1), records_s = sec(line.last);
        const double construct_s = std::chrono::duration<double>(t0 - tc).count(); // the core + every engine
        const double hold_s = tail ? std::chrono::duration<double>(tail->released - line.last).count() : 0.0;
        double search_s = 0.0, handback_s = 0.0, prep_s = 0.0, dev_s = 0.0, fetch_s = 0.0; // summed over the HIP
        for (auto* hip : hips) {                                                          // engines (concurrent)
            search_s += hip->searchSeconds();
            handback_s += hip->handbackSeconds();
            prep_s += hip->prepareSeconds();
            dev_s += hip->deviceSeconds();
            fetch_s += hip->fetchSeconds();
        }
        std::printf("{\"mode\": \"%s\", \"batch\": %zu, \"ranges\": %zu, \"cpu_engines\": %d, \"hip_engines\": %zu, "
                    "\"encode_s\": %.6f, \"records_s\": %.6f, \"tail_hold_s\": %.6f, \"drop_in_s\": %.6f, "
                    "\"hip_search_s\": %.6f, \"hip_handback_s\": %.6f, \"construct_s\": %.6f, "
                    "\"hip_prepare_s\": %.6f, \"hip_device_s\": %.6f, \"hip_fetch_s\": %.6f}\n",
                    batch ? "batch" : "ref", batch, targetGrid.items().size(), ncpu, hips.size(), encode_s, records_s,
                    hold_s, encode_s - hold_s, search_s, handback_s, construct_s, prep_s, dev_s, fetch_s);
        std::fflush(stdout);
    }
    for (auto* hip : hips) {
        try {
            hip->rethrowIfFailed(); // the failure of finalize(), on this thread
        } catch (const std::exception& exc) {
            std::fprintf(stderr, "HIP engine failed: %s (%zu ranges without a record)\n", exc.what(), hip->lostRanges());
            return 6;
        }
    }
    // the CPU engines' rejected mappings accumulate in the shared estimator (TransformEstimator2.hpp:59)
    rejected = estimator.rejectedMappings();
    uint64_t hip_ranges = 0;
    std::vector<uint64_t> per_engine;
    for (auto* hip : hips) {
        rejected += hip->rejectedMappings();
        hip_ranges += hip->searchedRanges();
        per_engine.push_back(hip->searchedRanges());
    }
    const uint64_t n_hip = hips.size();
    const std::vector<encode_item_t> encoded = batch ? batched : core.result().encoded;
    std::ofstream out(argv[9], std::ios::binary);
    out.write(reinterpret_cast<const char*>(encoded.data()), encoded.size() * sizeof(Frac::encode_item_t));
    out.write(reinterpret_cast<const char*>(&rejected), sizeof(rejected));
    out.write(reinterpret_cast<const char*>(&hip_ranges), sizeof(hip_ranges));
    out.write(reinterpret_cast<const char*>(per_engine.data()), per_engine.size() * sizeof(uint64_t));
    out.write(reinterpret_cast<const char*>(&n_hip), sizeof(n_hip));
    return out ? 0 : 5;
}

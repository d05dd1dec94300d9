// host_test.cpp — drives the C++ host layer (include/fracenc.hpp) the way a C++ caller of
// the reference would (Encoder2 → EncodingEngineCore2 → engines), on the committed fixtures,
// and writes the results to one binary file that tests/test_cpp_host.py compares with the
// reference goldens.  Usage: host_test <repo root> <output file>
#include "fracenc.hpp"

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <vector>

static std::vector<uint8_t> read_plane(const std::string& path, size_t n)
{
    std::vector<uint8_t> v(n);
    std::ifstream f(path, std::ios::binary);
    if (!f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)n))
        throw fracenc::Error("cannot read " + path);
    return v;
}

template <typename T>
static void put(std::ofstream& o, const T* p, size_t n)
{
    const uint64_t bytes = n * sizeof(T);
    o.write(reinterpret_cast<const char*>(&bytes), sizeof(bytes));
    o.write(reinterpret_cast<const char*>(p), (std::streamsize)bytes);
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        std::cerr << "usage: host_test <repo root> <output file>\n";
        return 2;
    }
    try {
        const std::string root = argv[1];
        const uint32_t W = 512, H = 512;
        const auto y = read_plane(root + "/tests/golden/lenna_y.u8", (size_t)W * H);
        std::ofstream out(argv[2], std::ios::binary);

        // 1. main.cpp:142-166: grids, then the engine core — two engines (contexts, streams)
        //    on GPU 0 claiming batches of 1,000 ranges
        const auto doms = fracenc::createUniformGrid(W, H, 16, 8);
        const auto rngs = fracenc::createUniformGrid(W, H, 8, 8);
        fracenc::Params p;
        fracenc::EncodingEngineCore core(p, {0, 0}, 1000);
        frac_stats st{};
        const auto t4 = core.encode(y.data(), W, H, W, doms, rngs, &st);
        put(out, t4.data(), t4.size());
        put(out, &st.rejected_mappings, 1);

        // 2. classifier on: categories left at -1, computed by the engines on the device
        fracenc::Params pc;
        pc.use_classifier = true;
        fracenc::EncodingEngineCore core_c(pc, {0}, 1500);
        const auto cls = core_c.encode(y.data(), W, H, W, doms, rngs, &st);
        put(out, cls.data(), cls.size());
        put(out, &st.rejected_mappings, 1);

        // 3. main.cpp:106-140: Quantizer over the frame's contrast / brightness, 5 / 7 bits
        double smin = 1e300, smax = -1e300, omin = 1e300, omax = -1e300;
        for (const auto& e : t4) {
            smin = std::min(smin, e.match.score.contrast);
            smax = std::max(smax, e.match.score.contrast);
            omin = std::min(omin, e.match.score.brightness);
            omax = std::max(omax, e.match.score.brightness);
        }
        fracenc::Quantizer<double> qs(smin, smax, 5), qo(omin, omax, 7);
        std::vector<uint64_t> codes;
        std::vector<double> values;
        for (const auto& e : t4) {
            codes.push_back(qs.quantized(e.match.score.contrast));
            values.push_back(qs.value(codes.back()));
        }
        for (const auto& e : t4) {
            codes.push_back(qo.quantized(e.match.score.brightness));
            values.push_back(qo.value(codes.back()));
        }
        put(out, codes.data(), codes.size());
        put(out, values.data(), values.size());

        // 4. Decoder2 (main.cpp:171-176) on the engine
        fracenc::Engine e(0, p);
        std::vector<uint8_t> plane((size_t)W * H, 0);
        const auto r = e.decode(t4, W, H, plane);
        put(out, plane.data(), plane.size());
        const int32_t it = r.first;
        put(out, &it, 1);
        put(out, &r.second, 1);
        // 5. ABI 9 frame streaming on one engine: three frames, each uploaded by setFrameAsync while the
        //    previous one's run is enqueued, the tuples of every frame fetched; beside them each frame's tuples
        //    from a synchronous setFrame + run
        std::vector<std::vector<uint8_t>> frames(3, y);
        for (uint32_t r = 0; r < H; ++r)
            for (uint32_t c = 0; c < W; ++c) {
                frames[1][(size_t)r * W + c] = y[(size_t)(H - 1 - r) * W + c];
                frames[2][(size_t)r * W + c] = y[(size_t)r * W + (W - 1 - c)];
            }
        std::vector<frac_tuple> sync_t(rngs.size() * frames.size()), async_t(sync_t.size());
        {
            fracenc::Engine s(0, p);
            s.setDomains(doms);
            for (size_t k = 0; k < frames.size(); ++k) {
                s.setFrame(frames[k].data(), W, H, W);
                s.setRanges(rngs.data(), rngs.size());
                s.run();
                s.fetchTuples(sync_t.data() + k * rngs.size());
            }
        }
        fracenc::Params pt = p;
        pt.timing = true;
        fracenc::Engine a(0, pt);
        a.setFrame(frames[0].data(), W, H, W);
        a.setDomains(doms);
        a.setRanges(rngs.data(), rngs.size());
        for (size_t k = 0; k < frames.size(); ++k) {
            a.setFrameAsync(frames[k].data(), W, H, W);
            a.run();
            a.fetchTuples(async_t.data() + k * rngs.size());
        }
        put(out, sync_t.data(), sync_t.size());
        put(out, async_t.data(), async_t.size());
        // 6. the per-run device times of those three runs (Params::timing)
        const auto hist = a.timingHistory();
        const uint64_t nh = hist.size();
        put(out, &nh, 1);
        // 7. the quadtree partition as 32-byte leaves (ABI 7)
        fracenc::Params pq;
        pq.use_classifier = true;
        fracenc::Engine q(0, pq);
        q.setFrame(y.data(), W, H, W);
        const auto leaves = q.encodeQuadtreeLeaves(16, 4, 4.0);
        put(out, leaves.data(), leaves.size());
        std::cout << "host_test: ok (" << core.engineCount() << " engines)\n";
        return 0;
    } catch (const std::exception& ex) {
        std::cerr << "host_test: " << ex.what() << "\n";
        return 1;
    }
}

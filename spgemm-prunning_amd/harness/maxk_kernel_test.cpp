// maxk_kernel_test -- the reference's kernel benchmark as a compiled consumer of the C ABI
// (include/maxk_hip.h; libmaxk_hip.so).  Restates ./maxk_kernel_test <graph>
// (kernels/main.cu:50-221) and its timing recipe SPMM_BASE::timing_body
// (kernels/spmm_base.h:34-61):
//   * the graph is <dir>/<graph>.indptr|.indices (raw int32, data.h:9-24); with no graph
//     argument every <dir>/*.indptr is run (main.cu:187-221);
//   * inputs from std::default_random_engine seeded 123 and U(0,1) (main.cu:74-97): edge
//     values, then (drawn and unused, as in the reference, so the stream lines up) the
//     V x 64 sparse-data and V x 256 dense buffers, then per k (16, 32, 64; main.cu:52-54,
//     111-117) each row's k distinct columns by std::sample and their U(0,1) values
//     (main.cu:122-133), scattered into the dense input (:135-146);
//   * the library SpMM (rocSPARSE here, cuSPARSE there) once on the first k's dense input,
//     10 warmup + 10 timed runs (spmm_cusparse.cu:35-51, main.cu:163-166);
//   * the MaxK forward SpGEMM and backward SSpMM, 4 warmup + 4 timed runs, wall clock around
//     a device synchronize (spmm_base.h:34-61); the backward takes the dense input as its
//     gradient, as the reference's SPMM_MAXK_BACKWARD does (main.cu:102-103);
//   * output: the reference's "num graph dim_origin dim_k kernel time(ms)" lines.
// The backward mode is the C ABI's "auto" rule (maxk_backward_mode_auto, with the graph's
// pull locality) unless --bwd names one; its per-graph plan is built before the timing, the
// analogue of the reference's .warp4 files.
//
// --graph-replay (r06): every timed MaxK call is captured once into a hipGraph and timed as one
// hipGraphLaunch + synchronize (the library SpMM too, when its calls capture), so the wall
// clock shows the kernels without the per-kernel launch cost of a multi-kernel op.
// Extra modes for testing through the C ABI alone:
//   --check            check_err (main.cu:19-48, disabled in the reference) of the forward
//                      against the library SpMM: error sum, "validation pass!" below 1e-3 mean;
//   --inputs DIR       read val.f32 [E], cbsr_val.f32 [V,k], cbsr_idx.u8 [V,k], grad.f32
//                      [V,dim] and optional row_div.f32 [V] instead of the random inputs;
//   --dump DIR         write y.f32 [V,dim] and gs.f32 [V,k] (forward and backward outputs).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dirent.h>
#include <fstream>
#include <functional>
#include <iostream>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include "maxk_hip.h"

namespace {

#define HIP_CHECK(call)                                                                   \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));        \
            std::exit(2);                                                                 \
        }                                                                                 \
    } while (0)
#define MAXK_CHECK(call)                                                                  \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_ != MAXK_OK) {                                                             \
            std::fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, maxk_last_error());   \
            std::exit(3);                                                                 \
        }                                                                                 \
    } while (0)

template <typename T>
std::vector<T> read_array(const std::string &path, bool required = true) {
    std::ifstream in(path, std::ios::binary);
    if (!in) {
        if (required) {
            std::fprintf(stderr, "cannot open %s\n", path.c_str());
            std::exit(1);
        }
        return {};
    }
    in.seekg(0, std::ios::end);
    const size_t bytes = (size_t)in.tellg();
    in.seekg(0, std::ios::beg);
    std::vector<T> v(bytes / sizeof(T));
    in.read(reinterpret_cast<char *>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
    return v;
}

template <typename T>
void write_array(const std::string &path, const std::vector<T> &v) {
    std::ofstream out(path, std::ios::binary);
    out.write(reinterpret_cast<const char *>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
}

// caller-owned device buffer
struct Buf {
    void *p = nullptr;
    size_t n = 0;
    Buf() = default;
    explicit Buf(size_t bytes) { alloc(bytes); }
    void alloc(size_t bytes) {
        release();
        n = bytes;
        HIP_CHECK(hipMalloc(&p, bytes ? bytes : 1));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~Buf() { release(); }
    Buf(const Buf &) = delete;
    Buf &operator=(const Buf &) = delete;
    template <typename T>
    T *as() const { return reinterpret_cast<T *>(p); }
};

template <typename T>
void upload(Buf &b, const std::vector<T> &v) {
    b.alloc(v.size() * sizeof(T));
    if (!v.empty()) HIP_CHECK(hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
}

template <typename T>
std::vector<T> download(const Buf &b, size_t count) {
    std::vector<T> v(count);
    if (count) HIP_CHECK(hipMemcpy(v.data(), b.p, count * sizeof(T), hipMemcpyDeviceToHost));
    return v;
}

// The stream every timed call launches on: the legacy default stream, or with --graph-replay
// a created one whose calls are captured into a hipGraph (r06).
hipStream_t g_stream = nullptr;
bool g_replay = false;

// SPMM_BASE::timing_body (spmm_base.h:34-61): `times` warmup runs, then `times` timed runs,
// each bracketed by a device synchronize; returns the mean in seconds.  --graph-replay: the
// call is captured once on g_stream into a hipGraph and each run is one hipGraphLaunch of it
// (the op's several kernels leave the host in one submission) -- the same wall clock around
// it.  A call that cannot be captured (the library's) runs as is; `replayed` says which.
double timing_body(const std::function<void()> &run, int times, bool *replayed = nullptr) {
    if (replayed) *replayed = false;
    if (g_replay) {
        HIP_CHECK(hipDeviceSynchronize());  // setup on the legacy stream (plans) has finished
        run();  // first call outside the capture (lazy one-time setup in the library)
        HIP_CHECK(hipStreamSynchronize(g_stream));
        hipGraph_t graph = nullptr;
        hipGraphExec_t exec = nullptr;
        bool ok = hipStreamBeginCapture(g_stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
        if (ok) {
            run();
            ok = hipStreamEndCapture(g_stream, &graph) == hipSuccess && graph != nullptr &&
                 hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) == hipSuccess;
        }
        if (ok) {
            for (int i = 0; i < times; ++i) HIP_CHECK(hipGraphLaunch(exec, g_stream));
            HIP_CHECK(hipStreamSynchronize(g_stream));
            double total = 0;
            for (int i = 0; i < times; ++i) {
                const auto t0 = std::chrono::system_clock::now();
                HIP_CHECK(hipGraphLaunch(exec, g_stream));
                HIP_CHECK(hipStreamSynchronize(g_stream));
                const auto t1 = std::chrono::system_clock::now();
                total += std::chrono::duration<double>(t1 - t0).count();
            }
            HIP_CHECK(hipGraphExecDestroy(exec));
            HIP_CHECK(hipGraphDestroy(graph));
            if (replayed) *replayed = true;
            return total / times;
        }
        (void)hipGetLastError();
        if (graph) (void)hipGraphDestroy(graph);
    }
    for (int i = 0; i < times; ++i) run();
    HIP_CHECK(hipDeviceSynchronize());
    double total = 0;
    for (int i = 0; i < times; ++i) {
        const auto t0 = std::chrono::system_clock::now();
        run();
        HIP_CHECK(hipDeviceSynchronize());
        const auto t1 = std::chrono::system_clock::now();
        total += std::chrono::duration<double>(t1 - t0).count();
    }
    return total / times;
}

struct Options {
    std::string dir = "../graphs/";  // main.cu:10
    std::string graph;
    std::vector<int> ks = {16, 32, 64};
    int dim = 256;
    std::string bwd = "auto";
    bool check = false;
    std::string inputs, dump;
    int runs = 4, lib_runs = 10;
};

const char *mode_name(int m) {
    switch (m) {
        case MAXK_BWD_PULL: return "pull";
        case MAXK_BWD_CSC: return "csc";
        case MAXK_BWD_HYBRID: return "hybrid";
        case MAXK_BWD_ATOMIC: return "atomic";
        case MAXK_BWD_BSORT: return "bsort";
        case MAXK_BWD_DENSE: return "dense";
    }
    return "?";
}

int mode_of(const std::string &s) {
    if (s == "pull") return MAXK_BWD_PULL;
    if (s == "csc") return MAXK_BWD_CSC;
    if (s == "hybrid") return MAXK_BWD_HYBRID;
    if (s == "atomic") return MAXK_BWD_ATOMIC;
    if (s == "bsort") return MAXK_BWD_BSORT;
    if (s == "dense") return MAXK_BWD_DENSE;
    return -1;
}

// The backward of one graph at width k: the per-graph plan (built once, untimed) and a run()
// that launches it through the C ABI on the default stream.
struct Backward {
    int mode = MAXK_BWD_CSC;
    Buf plan_a, plan_b, plan_c, plan_d, plan_e, ws;
    // hybrid
    Buf tile_list, tile_ent, bucket_ptr, bucket_tiles, ent_pull, off_ip, off_col, off_val,
        off_cp, off_eid;
    int64_t counts[3] = {0, 0, 0};
    int shift = 0, slices = 1;
    std::function<void()> run;
};

void build_backward(Backward &b, const Buf &ip, const Buf &ix, const Buf &val, const Buf &grad,
                    const Buf &row_div_b, const float *row_div, const Buf &sel, Buf &gs,
                    int64_t V, int64_t E, int D, int k) {
    const int32_t *rp = ip.as<int32_t>(), *ci = ix.as<int32_t>();
    const float *ev = val.as<float>(), *G = grad.as<float>();
    const uint8_t *S = sel.as<uint8_t>();
    float *out = gs.as<float>();
    (void)row_div_b;
    switch (b.mode) {
        case MAXK_BWD_PULL: {
            b.shift = maxk_pull_shift(k);
            b.slices = maxk_pull_slices(V, V, D, k);
            const int64_t nb = maxk_bucket_count(V, b.shift);
            b.plan_a.alloc((size_t)(b.slices * nb + 1) * 4);
            b.plan_b.alloc((size_t)E * 8);
            Buf pws(maxk_pull_plan_workspace_size(V, V, E, b.shift, b.slices));
            MAXK_CHECK(maxk_pull_plan(rp, ci, ev, V, V, E, b.shift, b.slices, b.plan_a.as<int32_t>(),
                                      b.plan_b.as<uint32_t>(), pws.p, pws.n, nullptr));
            HIP_CHECK(hipDeviceSynchronize());
            b.ws.alloc(maxk_sspmm_backward_pull_workspace_size(V, V, D, k, b.slices));
            b.run = [&b, G, row_div, S, out, V, E, D, k] {
                MAXK_CHECK(maxk_sspmm_backward_pull(G, row_div, S, b.plan_a.as<int32_t>(),
                                                    b.plan_b.as<uint32_t>(), b.shift, b.slices,
                                                    out, V, V, E, D, k, b.ws.p, b.ws.n, g_stream));
            };
            return;
        }
        case MAXK_BWD_HYBRID: {
            b.shift = maxk_pull_shift(k);
            b.slices = maxk_pull_slices(V, V, D, k);
            const int64_t nb = maxk_bucket_count(V, b.shift), nt = b.slices * nb;
            Buf tptr((size_t)(nt + 1) * 4), ent((size_t)E * 8);
            {
                Buf pws(maxk_pull_plan_workspace_size(V, V, E, b.shift, b.slices));
                MAXK_CHECK(maxk_pull_plan(rp, ci, ev, V, V, E, b.shift, b.slices,
                                          tptr.as<int32_t>(), ent.as<uint32_t>(), pws.p, pws.n,
                                          nullptr));
            }
            b.tile_list.alloc((size_t)nt * 4);
            b.tile_ent.alloc((size_t)(nt + 1) * 4);
            b.bucket_ptr.alloc((size_t)(nb + 1) * 4);
            b.bucket_tiles.alloc((size_t)nt * 4);
            b.ent_pull.alloc((size_t)E * 8);
            b.off_ip.alloc((size_t)(V + 1) * 4);
            b.off_col.alloc((size_t)E * 4);
            b.off_val.alloc((size_t)E * 4);
            Buf hws(maxk_hybrid_plan_workspace_size(V, V, E, b.shift, b.slices));
            MAXK_CHECK(maxk_hybrid_plan(rp, ci, ev, tptr.as<int32_t>(), ent.as<uint32_t>(), V, V, E,
                                        b.shift, b.slices, MAXK_HYBRID_DENSITY,
                                        b.tile_list.as<int32_t>(), b.tile_ent.as<int32_t>(),
                                        b.bucket_ptr.as<int32_t>(), b.bucket_tiles.as<int32_t>(),
                                        b.ent_pull.as<uint32_t>(), b.off_ip.as<int32_t>(),
                                        b.off_col.as<int32_t>(), b.off_val.as<float>(), b.counts,
                                        hws.p, hws.n, nullptr));
            b.off_cp.alloc((size_t)(V + 1) * 4);
            b.off_eid.alloc((size_t)std::max<int64_t>(b.counts[2], 1) * 4);
            Buf tws(maxk_transpose_plan_workspace_size(V, b.counts[2]));
            MAXK_CHECK(maxk_transpose_plan(b.off_col.as<int32_t>(), V, b.counts[2],
                                           b.off_cp.as<int32_t>(), b.off_eid.as<int32_t>(), tws.p,
                                           tws.n, nullptr));
            HIP_CHECK(hipDeviceSynchronize());
            b.ws.alloc(maxk_sspmm_backward_hybrid_workspace_size(V, V, b.counts[2], D, k, b.counts[0]));
            b.run = [&b, G, row_div, S, out, V, D, k] {
                MAXK_CHECK(maxk_sspmm_backward_hybrid(
                    G, row_div, S, b.tile_list.as<int32_t>(), b.tile_ent.as<int32_t>(),
                    (int32_t)b.counts[0], b.bucket_ptr.as<int32_t>(), b.bucket_tiles.as<int32_t>(),
                    b.ent_pull.as<uint32_t>(), b.counts[1], b.shift, b.slices,
                    b.off_ip.as<int32_t>(), b.off_col.as<int32_t>(), b.off_val.as<float>(),
                    b.counts[2], b.off_cp.as<int32_t>(), b.off_eid.as<int32_t>(), 0, out, V, V, D,
                    k, b.ws.p, b.ws.n, g_stream, nullptr, nullptr, nullptr));
            };
            return;
        }
        case MAXK_BWD_BSORT: {  // window-sorted two-phase, selectors gathered from the table
            b.shift = maxk_bucket_shift(k);
            const int64_t nb = maxk_bucket_count(V, b.shift);
            b.plan_a.alloc((size_t)(nb + 1) * 4);
            b.plan_b.alloc((size_t)E * 4);
            b.plan_c.alloc((size_t)E * 2);
            b.plan_d.alloc((size_t)E * 2);
            b.plan_e.alloc((size_t)E * 4);
            Buf pws(maxk_bsort_plan_workspace_size(V, E));
            MAXK_CHECK(maxk_bsort_plan(rp, ci, V, V, E, k, b.shift, b.plan_a.as<int32_t>(),
                                       b.plan_b.as<int32_t>(), b.plan_c.as<uint16_t>(),
                                       b.plan_d.as<uint16_t>(), b.plan_e.as<int32_t>(), pws.p,
                                       pws.n, nullptr));
            HIP_CHECK(hipDeviceSynchronize());
            b.ws.alloc(maxk_sspmm_backward_bsort_workspace_size(V, V, E, D, k));
            b.run = [&b, rp, ci, ev, G, row_div, S, out, V, E, D, k] {
                MAXK_CHECK(maxk_sspmm_backward_bsort(
                    rp, ci, ev, G, row_div, S, nullptr, b.plan_a.as<int32_t>(),
                    b.plan_b.as<int32_t>(), b.plan_c.as<uint16_t>(), b.plan_d.as<uint16_t>(),
                    b.plan_e.as<int32_t>(), b.shift, out, V, V, E, D, k, b.ws.p, b.ws.n, g_stream));
            };
            return;
        }
        case MAXK_BWD_DENSE: {  // k >= D / 2: dense G rows along the transpose
            b.plan_a.alloc((size_t)(V + 1) * 4);
            b.plan_b.alloc((size_t)E * 4);
            b.plan_c.alloc((size_t)E * 4);
            b.plan_d.alloc((size_t)E * 4);
            {
                Buf tws(maxk_transpose_plan_workspace_size(V, E));
                MAXK_CHECK(maxk_transpose_plan(ci, V, E, b.plan_a.as<int32_t>(),
                                               b.plan_b.as<int32_t>(), tws.p, tws.n, nullptr));
                MAXK_CHECK(maxk_dense_plan(rp, ev, b.plan_b.as<int32_t>(), V, E,
                                           b.plan_c.as<int32_t>(), b.plan_d.as<float>(), nullptr));
                HIP_CHECK(hipDeviceSynchronize());
            }
            b.ws.alloc(maxk_sspmm_backward_dense_workspace_size(V, V, E, D, k, 0));
            b.run = [&b, G, row_div, S, out, V, E, D, k] {
                MAXK_CHECK(maxk_sspmm_backward_dense(b.plan_a.as<int32_t>(), b.plan_c.as<int32_t>(),
                                                     b.plan_d.as<float>(), G, row_div, S, out, V,
                                                     V, E, D, k, 0, b.ws.p, b.ws.n, g_stream));
            };
            return;
        }
        case MAXK_BWD_ATOMIC: {
            b.ws.alloc(maxk_sspmm_backward_workspace_size(V, V, E, D, k, 0));
            b.run = [&b, rp, ci, ev, G, row_div, S, out, V, E, D, k] {
                MAXK_CHECK(maxk_sspmm_backward(rp, ci, ev, G, row_div, S, out, V, V, E, D, k, 0,
                                               b.ws.p, b.ws.n, g_stream));
            };
            return;
        }
        default: {  // csc
            b.plan_a.alloc((size_t)(V + 1) * 4);
            b.plan_b.alloc((size_t)E * 4);
            Buf tws(maxk_transpose_plan_workspace_size(V, E));
            MAXK_CHECK(maxk_transpose_plan(ci, V, E, b.plan_a.as<int32_t>(), b.plan_b.as<int32_t>(),
                                           tws.p, tws.n, nullptr));
            HIP_CHECK(hipDeviceSynchronize());
            b.ws.alloc(maxk_sspmm_backward_csc_workspace_size(V, V, E, D, k, 0));
            b.run = [&b, rp, ci, ev, G, row_div, S, out, V, E, D, k] {
                MAXK_CHECK(maxk_sspmm_backward_csc(rp, ci, ev, G, row_div, S, b.plan_a.as<int32_t>(),
                                                   b.plan_b.as<int32_t>(), out, V, V, E, D, k, 0,
                                                   b.ws.p, b.ws.n, g_stream));
            };
            return;
        }
    }
}

// check_err (main.cu:19-48): the error sum over all elements; pass below 1e-3 per element
double check_err(const std::vector<float> &out, const std::vector<float> &ref, bool &has_err) {
    double sum = 0;
    has_err = false;
    for (size_t i = 0; i < out.size(); ++i) {
        const double e = std::abs((double)out[i] - (double)ref[i]);
        sum += e;
        if (e > 0.1) has_err = true;
    }
    std::cout << "err sum = " << sum << "  ";
    std::cout << (sum / std::max<size_t>(out.size(), 1) < 0.001 ? "validation pass!" : "validation fail!")
              << std::endl;
    return sum;
}

int test_graph(const Options &o, const std::string &graph, int cur, int total) {
    const std::vector<int32_t> indptr = read_array<int32_t>(o.dir + "/" + graph + ".indptr");
    const std::vector<int32_t> indices = read_array<int32_t>(o.dir + "/" + graph + ".indices");
    if (indptr.empty()) {
        std::fprintf(stderr, "%s: empty indptr\n", graph.c_str());
        return 1;
    }
    const int64_t V = (int64_t)indptr.size() - 1, E = (int64_t)indices.size();
    const int D = o.dim;
    const int k_limit = 64;  // main.cu:54
    Buf ip, ix, val, y, ylib, dense, sv, ss, gs, grad, rdiv;
    upload(ip, indptr);
    upload(ix, indices);

    std::default_random_engine engine;  // main.cu:74-85
    engine.seed(123);
    std::uniform_real_distribution<float> rd(0, 1);
    std::vector<float> h_val;
    std::vector<float> h_rdiv;
    if (o.inputs.empty()) {
        h_val.resize((size_t)E);
        std::generate(h_val.begin(), h_val.end(), [&] { return rd(engine); });
        // drawn and unused (main.cu:96-97), so the per-k draws below line up with the reference
        for (int64_t i = 0; i < V * k_limit; ++i) (void)rd(engine);
        for (int64_t i = 0; i < V * D; ++i) (void)rd(engine);
    } else {
        h_val = read_array<float>(o.inputs + "/val.f32");
        h_rdiv = read_array<float>(o.inputs + "/row_div.f32", false);
        if ((int64_t)h_val.size() != E || (!h_rdiv.empty() && (int64_t)h_rdiv.size() != V)) {
            std::fprintf(stderr, "--inputs: val.f32 / row_div.f32 do not match the graph\n");
            return 1;
        }
    }
    upload(val, h_val);
    const float *row_div = nullptr;
    if (!h_rdiv.empty()) {
        upload(rdiv, h_rdiv);
        row_div = rdiv.as<float>();
    }
    y.alloc((size_t)V * D * 4);
    ylib.alloc((size_t)V * D * 4);
    std::vector<int> sequence(D);
    std::iota(sequence.begin(), sequence.end(), 0);

    std::cout << "num graph dim_origin dim_k kernel time(ms)" << std::endl;
    // the graph's locality for the "auto" rule (synchronous, once)
    double locality = -1;
    for (size_t n = 0; n < o.ks.size(); ++n) {
        const int k = o.ks[n];
        if (o.inputs.empty() && k > k_limit) break;  // main.cu:113-116
        if (k < 1 || k > D) {
            std::fprintf(stderr, "k=%d out of [1, %d]\n", k, D);
            return 1;
        }
        const std::string tag = std::to_string(cur) + "/" + std::to_string(total) + " " + graph +
                                " " + std::to_string(D) + " " + std::to_string(k);
        std::vector<float> h_sv((size_t)V * k), h_dense, h_grad;
        std::vector<uint8_t> h_ss((size_t)V * k);
        if (o.inputs.empty()) {
            std::vector<int> sample(k);
            for (int64_t i = 0; i < V; ++i) {  // main.cu:122-133
                std::sample(sequence.begin(), sequence.end(), sample.begin(), k, engine);
                for (int j = 0; j < k; ++j) {
                    h_sv[i * k + j] = rd(engine);
                    h_ss[i * k + j] = (uint8_t)sample[j];
                }
            }
        } else {
            h_sv = read_array<float>(o.inputs + "/cbsr_val.f32");
            h_ss = read_array<uint8_t>(o.inputs + "/cbsr_idx.u8");
            h_grad = read_array<float>(o.inputs + "/grad.f32");
            if ((int64_t)h_sv.size() != V * k || (int64_t)h_ss.size() != V * k ||
                (int64_t)h_grad.size() != V * D) {
                std::fprintf(stderr, "--inputs: CBSR / grad sizes do not match V=%lld k=%d D=%d\n",
                             (long long)V, k, D);
                return 1;
            }
        }
        h_dense.assign((size_t)V * D, 0.f);  // main.cu:135-146
        for (int64_t i = 0; i < V; ++i)
            for (int j = 0; j < k; ++j) h_dense[i * D + h_ss[i * k + j]] = h_sv[i * k + j];
        upload(sv, h_sv);
        upload(ss, h_ss);
        upload(dense, h_dense);
        // the reference's backward takes the dense input as its gradient (main.cu:102-103)
        if (h_grad.empty()) {
            grad.release();
        } else {
            upload(grad, h_grad);
        }
        const Buf &G = h_grad.empty() ? dense : grad;
        gs.alloc((size_t)V * k * 4);

        if (n == 0 || o.check) {  // library SpMM once (main.cu:163-166); again for --check
            maxk_dense_spmm_plan *plan = nullptr;
            MAXK_CHECK(maxk_dense_spmm_plan_create(&plan, ip.as<int32_t>(), ix.as<int32_t>(),
                                                   val.as<float>(), dense.as<float>(),
                                                   ylib.as<float>(), V, V, E, D, 0, nullptr));
            bool rep = false;
            const double t = timing_body([&] { MAXK_CHECK(maxk_dense_spmm_run(plan, g_stream)); },
                                         o.lib_runs, &rep);
            MAXK_CHECK(maxk_dense_spmm_plan_destroy(plan));
            if (n == 0) std::cout << tag << " cusparse " << t * 1000 << std::endl;
            if (g_replay) std::cerr << "# " << tag << " library SpMM graph-replayed " << rep << std::endl;
        }

        const size_t fws_b = maxk_spgemm_forward_workspace_size(V, V, E, D, k, 0);
        Buf fws(fws_b);
        auto fwd = [&] {
            MAXK_CHECK(maxk_spgemm_forward(ip.as<int32_t>(), ix.as<int32_t>(), val.as<float>(),
                                           sv.as<float>(), ss.as<uint8_t>(), row_div, y.as<float>(),
                                           V, V, E, D, k, 0, fws.p, fws.n, g_stream));
        };
        bool rep_f = false, rep_b = false;
        const double t_f = timing_body(fwd, o.runs, &rep_f);
        std::cout << tag << " maxk " << t_f * 1000 << std::endl;
        if (o.check) {
            bool has_err = false;
            std::vector<float> yo = download<float>(y, (size_t)V * D);
            std::vector<float> yr = download<float>(ylib, (size_t)V * D);
            if (row_div)
                for (int64_t i = 0; i < V; ++i)
                    for (int j = 0; j < D; ++j) yr[i * D + j] /= h_rdiv[i];
            check_err(yo, yr, has_err);
        }

        Backward b;
        b.mode = mode_of(o.bwd);
        if (b.mode < 0) {  // "auto": the C ABI's rule, with the graph's locality when it matters
            b.mode = maxk_backward_mode_auto(V, V, E, D, k, -1.0);
            if ((b.mode == MAXK_BWD_CSC || b.mode == MAXK_BWD_BSORT) && k % 4 == 0 && E > 0) {
                if (locality < 0) {
                    Buf lws(8);
                    MAXK_CHECK(maxk_pull_locality(ip.as<int32_t>(), ix.as<int32_t>(), V, E,
                                                  maxk_pull_shift(k), &locality, lws.p, lws.n,
                                                  nullptr));
                }
                b.mode = maxk_backward_mode_auto(V, V, E, D, k, locality);
            }
        }
        build_backward(b, ip, ix, val, G, rdiv, row_div, ss, gs, V, E, D, k);
        const double t_b = timing_body(b.run, o.runs, &rep_b);
        std::cout << tag << " maxk_backward " << t_b * 1000 << std::endl;
        std::cerr << "# " << tag << " backward mode " << mode_name(b.mode) << std::endl;
        if (g_replay)
            std::cerr << "# " << tag << " graph-replayed forward " << rep_f << " backward " << rep_b
                      << std::endl;
        if (!o.dump.empty()) {
            write_array(o.dump + "/y.f32", download<float>(y, (size_t)V * D));
            write_array(o.dump + "/gs.f32", download<float>(gs, (size_t)V * k));
        }
    }
    return 0;
}

std::vector<int> parse_ks(const std::string &s) {
    std::vector<int> ks;
    size_t p = 0;
    while (p < s.size()) {
        const size_t q = s.find(',', p);
        ks.push_back(std::atoi(s.substr(p, q == std::string::npos ? std::string::npos : q - p).c_str()));
        if (q == std::string::npos) break;
        p = q + 1;
    }
    return ks;
}

}  // namespace

int main(int argc, char **argv) {
    Options o;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "%s needs a value\n", a.c_str());
                std::exit(1);
            }
            return argv[++i];
        };
        if (a == "--dir") o.dir = next();
        else if (a == "--k") o.ks = parse_ks(next());
        else if (a == "--dim") o.dim = std::atoi(next().c_str());
        else if (a == "--bwd") o.bwd = next();
        else if (a == "--check") o.check = true;
        else if (a == "--inputs") o.inputs = next();
        else if (a == "--dump") o.dump = next();
        else if (a == "--runs") o.runs = std::atoi(next().c_str());
        else if (a == "--lib-runs") o.lib_runs = std::atoi(next().c_str());
        else if (a == "--graph-replay") g_replay = true;
        else if (a == "-h" || a == "--help") {
            std::printf("usage: %s [graph] [--dir DIR] [--k 16,32,64] [--dim 256] "
                        "[--bwd auto|pull|csc|hybrid|bsort|atomic|dense] [--check] [--runs 4] "
                        "[--inputs DIR] [--dump DIR] [--graph-replay]\n", argv[0]);
            return 0;
        } else if (!a.empty() && a[0] != '-') o.graph = a;
        else {
            std::fprintf(stderr, "unknown option %s\n", a.c_str());
            return 1;
        }
    }
    if (o.bwd != "auto" && mode_of(o.bwd) < 0) {
        std::fprintf(stderr, "--bwd must be auto, pull, csc, hybrid, bsort, atomic or dense\n");
        return 1;
    }
    if (maxk_device_count() < 1) {
        std::fprintf(stderr, "no HIP device\n");
        return 4;
    }
    if (g_replay) HIP_CHECK(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking));
    if (!o.graph.empty()) return test_graph(o, o.graph, 1, 1);
    // every <dir>/*.indptr (main.cu:197-217)
    std::vector<std::string> graphs;
    if (DIR *d = opendir(o.dir.c_str())) {
        while (dirent *e = readdir(d)) {
            const std::string n = e->d_name;
            if (n.size() > 7 && n.compare(n.size() - 7, 7, ".indptr") == 0)
                graphs.push_back(n.substr(0, n.size() - 7));
        }
        closedir(d);
    }
    std::sort(graphs.begin(), graphs.end());
    int rc = 0;
    for (size_t i = 0; i < graphs.size(); ++i) {
        rc |= test_graph(o, graphs[i], (int)i + 1, (int)graphs.size());
        HIP_CHECK(hipDeviceSynchronize());
    }
    return rc;
}

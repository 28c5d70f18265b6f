// Probe, not product: a stand-in for an RCCL collective's footprint on one GPU (VERDICT r05
// item 4), to run on a second stream beside a shard's aggregation kernels in tools/shard_probe.py
// --contention.  `channels` workgroups (RCCL runs one workgroup per channel, each resident on
// a CU for the collective's whole duration) copy `bytes` from src to dst -- with `reduce`, dst =
// src + src2 (a reduce-scatter step reads two buffers) -- in 64-KiB chunks, each workgroup
// holding its share to the pace of `gbps` GB/s overall (the bus bandwidth: the collective
// cannot move its bytes faster than the links deliver them) by waiting on the device's
// constant-rate wall clock between chunks.  The wait is a sleep loop, so an idle channel holds
// its CU slot but issues no memory traffic, as a channel waiting on its peer does.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/probe_lib/libpaced_copy.so tools/paced_copy.hip
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kThreads = 256;
constexpr int64_t kChunk = 64 << 10;

__global__ __launch_bounds__(kThreads) void paced_copy_kernel(const float4 *__restrict__ src,
                                                              const float4 *__restrict__ src2,
                                                              float4 *__restrict__ dst,
                                                              int64_t n16, double ticks_per_chunk) {
    const int64_t per_chunk = kChunk / 16;
    const int64_t n_chunks = (n16 + per_chunk - 1) / per_chunk;
    const uint64_t t0 = wall_clock64();
    int64_t done = 0;
    for (int64_t c = blockIdx.x; c < n_chunks; c += gridDim.x, ++done) {
        // pace: this workgroup's done-th chunk may start at t0 + done * ticks_per_chunk
        const uint64_t start = t0 + (uint64_t)(done * ticks_per_chunk);
        while (wall_clock64() < start) __builtin_amdgcn_s_sleep(8);
        const int64_t lo = c * per_chunk;
        const int64_t hi = lo + per_chunk < n16 ? lo + per_chunk : n16;
        for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
            float4 v = src[i];
            if (src2) {
                const float4 w = src2[i];
                v.x += w.x;
                v.y += w.y;
                v.z += w.z;
                v.w += w.w;
            }
            dst[i] = v;
        }
    }
}

}  // namespace

// bytes: multiple of 16; gbps <= 0: unpaced.  Returns 0, or the HIP error code.
extern "C" int paced_copy(const void *src, const void *src2, void *dst, int64_t bytes,
                          int channels, double gbps, void *stream) {
    int dev = 0, rate_khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess)
        return 1;
    const int64_t n16 = bytes / 16;
    const int64_t n_chunks = (n16 + kChunk / 16 - 1) / (kChunk / 16);
    // each channel moves n_chunks / channels chunks over bytes / gbps seconds
    const double secs_per_chunk_per_channel =
        gbps > 0 ? (double)kChunk * channels / (gbps * 1e9) : 0.0;
    const double ticks = secs_per_chunk_per_channel * rate_khz * 1e3;
    const int grid = channels < n_chunks ? channels : (int)(n_chunks > 0 ? n_chunks : 1);
    hipLaunchKernelGGL(paced_copy_kernel, dim3(grid), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const float4 *>(src), reinterpret_cast<const float4 *>(src2),
                       reinterpret_cast<float4 *>(dst), n16, ticks);
    return (int)hipGetLastError();
}

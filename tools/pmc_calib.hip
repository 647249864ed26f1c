// tools/pmc_calib.hip -- calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the
// access patterns of the MPH kernels (MI355X_MICROARCH.md: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
//
// Each kernel moves a known number of bytes through access patterns like those of the hot path:
//   stream_read16   coalesced 16-B loads (the guide's calibrated case: FETCH_SIZE = bytes / 2)
//   gather16        random 16-B loads (pass B's 32-B records are two of these per neighbour)
//   gather48        random 48-B records, three 16-B loads at consecutive addresses (pass A)
//   gather8         random 8-B loads
//   stream_write16  coalesced 16-B stores
//   scatter4_ell    4-B stores into ELL rows [tile][k][lane] with a per-lane row length, as
//                   k_neighbors writes the neighbour list
// over arrays far larger than the 256 MiB Infinity Cache, so the random patterns miss on-die.
// Prints one JSON line with the requested bytes and the 64-B line count of every kernel;
// tools/pmc_calib.py sets them against the counters of separate --pmc passes.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/pmc_calib tools/pmc_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(e)                                                                         \
    do {                                                                              \
        hipError_t _e = (e);                                                          \
        if (_e != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s: %s\n", #e, hipGetErrorString(_e));              \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

__device__ __forceinline__ unsigned long long mix(unsigned long long x)
{
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ void k_stream_read16(const double2* __restrict__ a, size_t n, double* __restrict__ sink)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) sink[0] = s;   // keep the loads
}

__global__ void k_gather16(const double2* __restrict__ a, size_t nrec, size_t n, double* __restrict__ sink)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2 v = a[mix(i) % nrec];
    if (v.x + v.y == 12345.678) sink[0] = v.x;
}

__global__ void k_gather48(const double2* __restrict__ a, size_t nrec, size_t n, double* __restrict__ sink)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2* q = a + 3 * (mix(i) % nrec);
    const double2 u = q[0], v = q[1], w = q[2];
    if (u.x + v.y + w.x == 12345.678) sink[0] = u.y;
}

__global__ void k_gather8(const double* __restrict__ a, size_t nrec, size_t n, double* __restrict__ sink)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = a[mix(i) % nrec];
    if (v == 12345.678) sink[0] = v;
}

__global__ void k_stream_write16(double2* __restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_double2((double)i, 1.0);
}

// rows of `len(lane)` 4-byte entries, entry k of a lane at [tile][k][lane] (64 lanes per tile),
// row length 64..80 varying per lane like NeighborCount; stores in k order, as the search does
__global__ void k_scatter4_ell(int* __restrict__ a, size_t ntile, int kmax)
{
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= ntile * 64) return;
    const int len = 64 + (int)(mix(i) % 17);
    int* row = a + (i >> 6) * (size_t)(64 * kmax) + (i & 63);
    for (int k = 0; k < len; ++k) row[(size_t)k * 64] = (int)i + k;
}

int main()
{
    const size_t big = 4ull << 30;                       // 4 GiB arrays: far beyond the 256 MiB MALL
    const size_t n_stream = (2ull << 30) / 16;           // 2 GiB streamed
    const size_t n_gather = 1ull << 25;                  // 33.5 M random accesses
    const size_t ntile = (1ull << 22) / 64;              // 4.2 M rows of the ELL pattern
    const int kmax = 512;
    char* buf;
    double* sink;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 0, big));
    int* ell;
    const size_t ell_bytes = ntile * 64 * (size_t)kmax * 4;
    CK(hipMalloc(&ell, ell_bytes));
    CK(hipDeviceSynchronize());
    const int t = 256;
    const double2* a2 = (const double2*)buf;
    for (int rep = 0; rep < 2; ++rep) {   // rep 0 warms up; the PMC summary averages both launches
        hipLaunchKernelGGL(k_stream_read16, dim3(16384), dim3(t), 0, 0, a2, n_stream, sink);
        hipLaunchKernelGGL(k_gather16, dim3((n_gather + t - 1) / t), dim3(t), 0, 0, a2, big / 16, n_gather, sink);
        hipLaunchKernelGGL(k_gather48, dim3((n_gather + t - 1) / t), dim3(t), 0, 0, a2, big / 48, n_gather, sink);
        hipLaunchKernelGGL(k_gather8, dim3((n_gather + t - 1) / t), dim3(t), 0, 0, (const double*)buf, big / 8,
                           n_gather, sink);
        hipLaunchKernelGGL(k_stream_write16, dim3(16384), dim3(t), 0, 0, (double2*)buf, n_stream);
        hipLaunchKernelGGL(k_scatter4_ell, dim3((ntile * 64 + t - 1) / t), dim3(t), 0, 0, ell, ntile, kmax);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
    }
    // requested bytes and 64-B lines touched per launch (random accesses: one line each)
    const double ell_entries = (double)ntile * 64 * 72.0;   // mean row length (64 + 0..16)
    std::printf("{\"stream_read16\": {\"bytes\": %zu, \"lines64\": %zu}, "
                "\"gather16\": {\"bytes\": %zu, \"lines64\": %zu}, "
                "\"gather48\": {\"bytes\": %zu, \"lines64_min\": %zu, \"lines64_max\": %zu}, "
                "\"gather8\": {\"bytes\": %zu, \"lines64\": %zu}, "
                "\"stream_write16\": {\"bytes\": %zu, \"lines64\": %zu}, "
                "\"scatter4_ell\": {\"bytes\": %.0f, \"lines64\": %.0f}}\n",
                n_stream * 16, n_stream * 16 / 64, n_gather * 16, n_gather, n_gather * 48, n_gather,
                2 * n_gather, n_gather * 8, n_gather, n_stream * 16, n_stream * 16 / 64, ell_entries * 4,
                ell_entries * 4 / 64);
    CK(hipFree(buf));
    CK(hipFree(ell));
    CK(hipFree(sink));
    return 0;
}

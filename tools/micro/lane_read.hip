// Microbenchmark: the scan's memory access pattern without the automaton work.
// (a) per-lane contiguous ranges read right-to-left in aligned 64-byte blocks (one block prefetched)
// (b) the same ranges read left-to-right
// (c) a fully coalesced stream (lane i reads 16 B at i, i+64*16, ...)
// (d) the same stream read 8 B and 4 B per lane (the record / queue loads of the sparse kernels)
// Every kernel reads exactly `bytes` per launch: tools/pmc_traffic.py turns their FETCH_SIZE into one
// correction factor per access pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(512) void k_lane_rev(const uint4* __restrict__ p, uint64_t bytes_per_lane, uint64_t n_lanes,
                                                  uint32_t* __restrict__ out) {
    const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (c >= n_lanes) return;
    const uint64_t b_lo = c * bytes_per_lane / 64, b_hi = (c + 1) * bytes_per_lane / 64 - 1;
    uint32_t acc = 0;
    uint4 n0 = p[4 * b_hi], n1 = p[4 * b_hi + 1], n2 = p[4 * b_hi + 2], n3 = p[4 * b_hi + 3];
    for (uint64_t b = b_hi; b + 1 > b_lo; --b) {
        const uint4 w0 = n0, w1 = n1, w2 = n2, w3 = n3;
        if (b > b_lo) {
            n0 = p[4 * (b - 1)];
            n1 = p[4 * (b - 1) + 1];
            n2 = p[4 * (b - 1) + 2];
            n3 = p[4 * (b - 1) + 3];
        }
        acc ^= w0.x ^ w0.y ^ w0.z ^ w0.w ^ w1.x ^ w1.y ^ w1.z ^ w1.w ^ w2.x ^ w2.y ^ w2.z ^ w2.w ^ w3.x ^ w3.y ^ w3.z ^ w3.w;
    }
    out[c] = acc;
}

__global__ __launch_bounds__(512) void k_lane_fwd(const uint4* __restrict__ p, uint64_t bytes_per_lane, uint64_t n_lanes,
                                                  uint32_t* __restrict__ out) {
    const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (c >= n_lanes) return;
    const uint64_t b_lo = c * bytes_per_lane / 64, b_hi = (c + 1) * bytes_per_lane / 64;
    uint32_t acc = 0;
    uint4 n0 = p[4 * b_lo], n1 = p[4 * b_lo + 1], n2 = p[4 * b_lo + 2], n3 = p[4 * b_lo + 3];
    for (uint64_t b = b_lo; b < b_hi; ++b) {
        const uint4 w0 = n0, w1 = n1, w2 = n2, w3 = n3;
        if (b + 1 < b_hi) {
            n0 = p[4 * (b + 1)];
            n1 = p[4 * (b + 1) + 1];
            n2 = p[4 * (b + 1) + 2];
            n3 = p[4 * (b + 1) + 3];
        }
        acc ^= w0.x ^ w0.y ^ w0.z ^ w0.w ^ w1.x ^ w1.y ^ w1.z ^ w1.w ^ w2.x ^ w2.y ^ w2.z ^ w2.w ^ w3.x ^ w3.y ^ w3.z ^ w3.w;
    }
    out[c] = acc;
}

__global__ __launch_bounds__(256) void k_coalesced(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 w = p[i];
        acc ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <class T>
__device__ __forceinline__ void k_stream(const T* __restrict__ p, uint64_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        acc ^= (uint32_t)p[i] ^ (uint32_t)((uint64_t)p[i] >> 16);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ __launch_bounds__(256) void k_stream8(const uint64_t* __restrict__ p, uint64_t n, uint32_t* __restrict__ out) {
    k_stream<uint64_t>(p, n, out);
}
__global__ __launch_bounds__(256) void k_stream4(const uint32_t* __restrict__ p, uint64_t n, uint32_t* __restrict__ out) {
    k_stream<uint32_t>(p, n, out);
}

// (e) per-lane forward walks of short runs of 16-byte records, the runs of neighbouring lanes adjacent
//     (k_select's SelRec walk over a lane's matched pairs: ~6 records per lane, one-ahead prefetch)
__global__ __launch_bounds__(256) void k_walk16(const uint4* __restrict__ p, uint64_t recs_per_lane, uint64_t n_lanes,
                                                uint32_t* __restrict__ out) {
    const uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (c >= n_lanes) return;
    const uint64_t r0 = c * recs_per_lane, r1 = r0 + recs_per_lane;
    uint32_t acc = 0;
    uint4 nx = p[r0];
    for (uint64_t r = r0; r < r1; ++r) {
        const uint4 w = nx;
        if (r + 1 < r1) nx = p[r + 1];
        acc ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    out[c] = acc;
}

// (f) 16-byte records in a scattered order, every record once (a multiplicative permutation: the
//     sparse kernels' gathers of event / pair records and text windows)
__global__ __launch_bounds__(256) void k_gather16(const uint4* __restrict__ p, uint64_t n16, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint4 w = p[(i * 2654435761ull) % n16];
        acc ^= w.x ^ w.y ^ w.z ^ w.w;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    const uint64_t bytes = 1200ull << 20;
    uint4* d;
    uint32_t* o;
    if (hipMalloc(&d, bytes + 4096) != hipSuccess || hipMalloc(&o, 64 << 20) != hipSuccess) return 1;
    (void)hipMemset(d, 1, bytes + 4096);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (uint64_t bpl : {512ull, 1024ull, 2048ull}) {
        const uint64_t lanes = bytes / bpl;
        for (int dir = 0; dir < 2; ++dir) {
            float best = 1e9;
            for (int it = 0; it < 6; ++it) {
                (void)hipEventRecord(a);
                if (dir == 0) k_lane_rev<<<(lanes + 511) / 512, 512>>>(d, bpl, lanes, o);
                else k_lane_fwd<<<(lanes + 511) / 512, 512>>>(d, bpl, lanes, o);
                (void)hipEventRecord(b);
                (void)hipEventSynchronize(b);
                float ms;
                (void)hipEventElapsedTime(&ms, a, b);
                if (it) best = ms < best ? ms : best;
            }
            printf("per-lane %s %4llu B/lane: %.3f ms  %.0f GB/s\n", dir ? "fwd" : "rev", (unsigned long long)bpl, best,
                   bytes / best / 1e6);
        }
    }
    float best = 1e9;
    for (int it = 0; it < 6; ++it) {
        (void)hipEventRecord(a);
        k_coalesced<<<256 * 8, 256>>>(d, bytes / 16, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (it) best = ms < best ? ms : best;
    }
    printf("coalesced: %.3f ms  %.0f GB/s\n", best, bytes / best / 1e6);
    for (int w : {8, 4}) {
        best = 1e9;
        for (int it = 0; it < 6; ++it) {
            (void)hipEventRecord(a);
            if (w == 8) k_stream8<<<256 * 8, 256>>>(reinterpret_cast<const uint64_t*>(d), bytes / 8, o);
            else k_stream4<<<256 * 8, 256>>>(reinterpret_cast<const uint32_t*>(d), bytes / 4, o);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            if (it) best = ms < best ? ms : best;
        }
        printf("stream %d B/lane: %.3f ms  %.0f GB/s\n", w, best, bytes / best / 1e6);
    }
    {
        const uint64_t rpl = 6, lanes = bytes / 16 / rpl;
        best = 1e9;
        for (int it = 0; it < 6; ++it) {
            (void)hipEventRecord(a);
            k_walk16<<<(lanes + 255) / 256, 256>>>(d, rpl, lanes, o);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            if (it) best = ms < best ? ms : best;
        }
        printf("walk16 (6 records/lane): %.3f ms  %.0f GB/s\n", best, lanes * rpl * 16 / best / 1e6);
    }
    best = 1e9;
    for (int it = 0; it < 6; ++it) {
        (void)hipEventRecord(a);
        k_gather16<<<256 * 8, 256>>>(d, bytes / 16, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        if (it) best = ms < best ? ms : best;
    }
    printf("gather16: %.3f ms  %.0f GB/s\n", best, bytes / best / 1e6);
    return 0;
}

// Calibration of the LDS PMC counters (SQ_LDS_IDX_ACTIVE, SQ_LDS_BANK_CONFLICT) on known cycle counts,
// so that k_scan's LDS-array cycles per byte can be read off its counters (bench.py roofline_compute).
// Per MI355X_MICROARCH.md (LDS table): a ds_read_b32 wave-instruction is two 32-lane groups, one LDS
// cycle each when conflict-free; each extra distinct dword on a busy bank adds a cycle.
//   k_lds<0>: conflict-free (lane l of a group reads dword l)          -> 2 cycles per instruction
//   k_lds<1>: 2-way (lane l reads dword 2l: lanes l, l+16 share a bank) -> 4 cycles per instruction
//   k_lds<3>: 4-way (dword 4l)                                          -> 8 cycles per instruction
// Every workgroup: 256 threads, READS ds_read_b32 per thread; 2048 workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int READS = 4096;

template <int MODE>
__global__ __launch_bounds__(256) void k_lds(uint32_t* __restrict__ out) {
    __shared__ uint32_t s[8192];
    for (int i = threadIdx.x; i < 8192; i += 256) s[i] = i * 2654435761u;
    __syncthreads();
    const int lane = threadIdx.x & 31;
    const int stride = MODE == 0 ? 1 : MODE == 1 ? 2 : 4;
    uint32_t acc = 0, a = (uint32_t)(lane * stride) & 0x1fffu;
#pragma unroll 16
    for (int i = 0; i < READS; ++i) {
        acc += *reinterpret_cast<volatile uint32_t*>(&s[a]);
        a = (a + 256u) & 0x1fffu;                 // the next 256-dword row: same banks, new dwords
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const int blocks = 2048;
    uint32_t* d;
    if (hipMalloc(&d, (size_t)blocks * 256 * 4) != hipSuccess) return 1;
    for (int rep = 0; rep < 3; ++rep) {
        k_lds<0><<<blocks, 256>>>(d);
        k_lds<1><<<blocks, 256>>>(d);
        k_lds<3><<<blocks, 256>>>(d);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"waves_per_launch\": %d, \"reads_per_wave\": %d, \"cycles_per_read\": {\"k_lds<0>\": 2, \"k_lds<1>\": 4, "
           "\"k_lds<3>\": 8}}\n", blocks * 4, READS);
    (void)hipFree(d);
    return 0;
}

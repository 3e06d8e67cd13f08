// Optional NER detector (BASELINE config 5): BERT-base token classification, bf16 on
// the MI355X matrix cores.  A PERSON_NAME detector the reference only hints at (the "full name / your
// name" hotword of main_service/dlp_config.yaml:170 has no detector behind it).
//
// C-ABI (plain device pointers, torch not involved; all calls enqueue on `stream` and return):
//   ner_gemm       C[M,N] = A[M,K] . W[N,K]^T + bias  (+ exact GELU | + residual)   bf16 in/out, f32 accumulate
//   ner_layernorm  y = LN(x) * gamma + beta  per row                                 bf16 in/out, f32 math
//   ner_embed      LN(word[id] + pos[s] + type[0])                                    -> bf16 hidden
//   ner_attention  softmax(Q K^T / sqrt(d) + mask) V per (sequence, head) from the fused QKV rows
//   ner_classify   logits[M, L] = H . Wc^T + bc                                       f32 out
//
// ner_gemm is the dense contraction: 128x128 output tiles per 256-thread workgroup, each wavefront a
// 64x64 quarter as 2x2 v_mfma_f32_32x32x16_bf16 tiles, K DMA'd global -> LDS in 64-wide slabs
// (global_load_lds, XOR-swizzled 16-byte chunks).  Operands are K-contiguous (activations row-major,
// nn.Linear weights [out, in]), which is exactly the MFMA's A / B lane map: lane l holds
// A[row l&31][k 8(l>>5) .. +7] and W[col l&31][same k] -- no transposes anywhere.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {      // round to nearest even (NaN kept quiet)
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// exact (erf) GELU with erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16 output
// rounding): one reciprocal, one exp, five FMAs and no branches -- ocml's erff branches per lane, which
// made the FFN-up epilogue a sizeable part of that GEMM
__device__ __forceinline__ float gelu_erf(float v) {
    const float x = v * 0.70710678118654752f, ax = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
    const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                             0.254829592f);
    const float y = 1.f - p * __expf(-ax * ax);
    return 0.5f * v * (1.f + copysignf(y, x));
}

constexpr int GB_M = 128, GB_N = 128, GB_K = 64;
constexpr int32_t CLS_ID = 101, SEP_ID = 102, PAD_ID = 0;     // (ner.py CLS, SEP, PAD)
constexpr int G_THREADS = 256;
#ifndef GEMM_PIPE
#define GEMM_PIPE 1         // k_gemm2 (double-buffered slabs); 0 = the single-buffer k_gemm
#endif
#ifndef GEMM_MF
#define GEMM_MF 1           // k_gemm2 MFMA shape: 0 = 32x32x16, 1 = 16x16x32
#endif
#ifndef GEMM_NB
#define GEMM_NB 2           // k_gemm2 LDS slab buffers: 2 (one slab in flight) or 3 (two, counted vmcnt)
#endif
#ifndef GEMM_PRIO
#define GEMM_PRIO 1         // raise the wave priority over each MFMA block (s_setprio)
#endif
#ifndef GEMM_BIG
#define GEMM_BIG 0          // allow the 256-row k_gemm2 tiles
#endif

enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RESID = 2 };

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// C = A . W^T + bias (+ epilogue).  A [M, K], W [N, K], C / R [M, N] bf16; bias f32 [N].
// Requires M % 128 == 0, N % 128 == 0, K % 64 == 0 (the host pads M).
//
// Per 64-wide K step the workgroup DMAs both 128 x 64 operand slabs straight into LDS
// (global_load_lds, 16 B per lane: no staging registers), then each wavefront runs 4 k-steps of
// 2 x 2 MFMAs on its 64 x 64 quarter.  LDS rows are 128 B with the 16-byte chunks XOR-swizzled by
// (row & 7) -- chunk c of row r is stored at position c ^ (r & 7) -- so the fragment reads of 8
// consecutive rows (one ds_read_b128 lane group) hit 8 different 16-byte bank groups; the swizzle is
// applied on the per-lane GLOBAL address, since an LDS-DMA writes lane l at base + 16 l.  One LDS
// buffer (32 KiB) and two barriers per step: latency is hidden by 3-4 workgroups per CU.
template <int EPI>
__global__ __launch_bounds__(G_THREADS) void k_gemm(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
                                                    const float* __restrict__ bias, const uint16_t* __restrict__ R,
                                                    uint16_t* __restrict__ C, int M, int N, int K) {
    __shared__ __attribute__((aligned(16))) uint16_t smem[(GB_M + GB_N) * GB_K];
    uint16_t* sA = smem;
    uint16_t* sB = smem + GB_M * GB_K;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-aware tile order (bijective): workgroups are dealt to the 8 XCDs round robin, so give each
    // XCD a contiguous run of tile ids -- the N tiles of one M row-block share their A rows in its L2
    const int tiles_n = N / GB_N;
    const int nwg = (int)gridDim.x, orig = (int)blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int tm = bid / tiles_n, tn = bid % tiles_n;
    const int m0 = tm * GB_M, n0 = tn * GB_N;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    // this lane's source rows / swizzled chunks for its 4 DMA instructions per operand
    const uint16_t* srcA[4];
    const uint16_t* srcB[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = (i * 4 + wave) * 64 + lane, row = q >> 3, pos = q & 7;
        const int col = 8 * (pos ^ (row & 7));
        srcA[i] = A + (size_t)(m0 + row) * K + col;
        srcB[i] = W + (size_t)(n0 + row) * K + col;
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    const int r = lane & 31, h = lane >> 5;
    for (int k0 = 0; k0 < K; k0 += GB_K) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int blk = (i * 4 + wave) * 64 * 8;      // this wave-instruction's 1 KiB of LDS
            __builtin_amdgcn_global_load_lds((gptr_t)(srcA[i] + k0), (lptr_t)(sA + blk), 16, 0, 0);
            __builtin_amdgcn_global_load_lds((gptr_t)(srcB[i] + k0), (lptr_t)(sB + blk), 16, 0, 0);
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < GB_K / 16; ++ks) {
            bf16x8 fa[2], fb[2];
            const int c = 2 * ks + h;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int ra = wm + 32 * i + r, rb = wn + 32 * i + r;
                fa[i] = *reinterpret_cast<const bf16x8*>(sA + ra * GB_K + 8 * (c ^ (ra & 7)));
                fb[i] = *reinterpret_cast<const bf16x8*>(sB + rb * GB_K + 8 * (c ^ (rb & 7)));
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue through LDS (the K loop left it free: 32 KiB), 64 rows at a time: the two wavefronts
    // holding those rows store their accumulators as a row-major f32 [64][128] image (C/D map of
    // 32x32x16: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)); then every thread
    // finishes 8-column chunks with 16-byte loads of the residual and 16-byte stores of C
    float* sC = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        if ((wave >> 1) == half) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int reg = 0; reg < 16; ++reg) {
                        const int row = 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                        sC[row * GB_N + wn + 32 * j + r] = acc[i][j][reg];
                    }
        }
        __syncthreads();
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int q = tid + t * G_THREADS, row = q >> 4, c8 = (q & 15) * 8;
            const float4 x0 = *reinterpret_cast<const float4*>(sC + row * GB_N + c8);
            const float4 x1 = *reinterpret_cast<const float4*>(sC + row * GB_N + c8 + 4);
            float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
            const int grow = m0 + 64 * half + row, gcol = n0 + c8;
            if (bias) {
                const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol);
                const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol + 4);
                v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
                v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
            }
            if (EPI == EPI_GELU) {
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
            } else if (EPI == EPI_RESID) {
                const uint4 rr = *reinterpret_cast<const uint4*>(R + (size_t)grow * N + gcol);
                const uint32_t rw[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    v[2 * e] += bf2f((uint16_t)(rw[e] & 0xffffu));
                    v[2 * e + 1] += bf2f((uint16_t)(rw[e] >> 16));
                }
            }
            uint4 o;
            o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
            o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
            *reinterpret_cast<uint4*>(C + (size_t)grow * N + gcol) = o;
        }
        __syncthreads();
    }
    (void)M;
}

// Epilogue of one 64-row group: the accumulators of the two wavefronts owning rows [64 g, 64 g + 64) are
// written to LDS as a row-major f32 [64][128] image by the caller; every thread then finishes 8-column
// chunks (bias, GELU / residual) with 16-byte loads of the residual and 16-byte stores of C.
template <int EPI, int NT, int ROWS>
__device__ __forceinline__ void gemm_finish(const float* sC, const float* bias, const uint16_t* R, uint16_t* C,
                                            int grow0, int n0, int N) {
    const int tid = threadIdx.x;
    __syncthreads();
#pragma unroll
    for (int t = 0; t < ROWS * 16 / NT; ++t) {
        const int q = tid + t * NT, row = q >> 4, c8 = (q & 15) * 8;
        const float4 x0 = *reinterpret_cast<const float4*>(sC + row * GB_N + c8);
        const float4 x1 = *reinterpret_cast<const float4*>(sC + row * GB_N + c8 + 4);
        float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        const int grow = grow0 + row, gcol = n0 + c8;
        if (bias) {
            const float4 b0 = *reinterpret_cast<const float4*>(bias + gcol);
            const float4 b1 = *reinterpret_cast<const float4*>(bias + gcol + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        if (EPI == EPI_GELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = gelu_erf(v[e]);
        } else if (EPI == EPI_RESID) {
            const uint4 rr = *reinterpret_cast<const uint4*>(R + (size_t)grow * N + gcol);
            const uint32_t rw[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[2 * e] += bf2f((uint16_t)(rw[e] & 0xffffu));
                v[2 * e + 1] += bf2f((uint16_t)(rw[e] >> 16));
            }
        }
        uint4 o;
        o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        o.z = (uint32_t)f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16);
        o.w = (uint32_t)f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16);
        *reinterpret_cast<uint4*>(C + (size_t)grow * N + gcol) = o;
    }
    __syncthreads();
}

// The pipelined form: BM x 128 output tiles (BM = 256: 8 wavefronts, BM = 128: 4), each wavefront a
// 64 x 64 block as 2 x 2 v_mfma_f32_32x32x16_bf16, and TWO LDS slab buffers -- the DMA of K-slab k+1
// (global_load_lds, 16 B per lane, source-swizzled as k_gemm) is issued before the MFMAs of slab k, so
// it runs under them, and one barrier per slab both retires it and frees slab k's buffer for slab k+2.
// BM = 256 for the N >= 2304 projections (>= 576 tiles, one 96 KiB workgroup per CU), BM = 128 for
// N = 768 (384 tiles, 64 KiB, two per CU).  All LDS is one __shared__ array (a second one would make
// hipcc drain the DMA queue before every first ds_read, cdna_hip_programming.md §5 item 4(a)).
template <int EPI, int BM, int MF, int NB>
__global__ __launch_bounds__(BM * 2) void k_gemm2(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
                                                  const float* __restrict__ bias, const uint16_t* __restrict__ R,
                                                  uint16_t* __restrict__ C, int M, int N, int K) {
    constexpr int NW = BM / 32, NT = NW * 64;
    constexpr int SA = BM * GB_K, SB = GB_N * GB_K;           // slab elements
    constexpr int IA = (SA * 2 / 1024) / NW, IB = (SB * 2 / 1024) / NW;   // 1 KiB DMA instructions per wave
    static_assert(IA * NW * 512 == SA && IB * NW * 512 == SB, "slabs are whole 1 KiB DMA instructions per wave");
    __shared__ __attribute__((aligned(16))) uint16_t smem[NB * (SA + SB)];
    // epilogue rows per pass: as many 64-row groups of the f32 [rows][128] image as the slab buffers hold
    constexpr int EG_FIT = (NB * (SA + SB) * 2) / (GB_N * 4) / 64 * 64;
    constexpr int EG = BM <= EG_FIT ? BM : BM / 2 <= EG_FIT ? BM / 2 : 64;
    static_assert(EG >= 64 && BM % EG == 0, "epilogue group");
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tiles_n = N / GB_N;
    const int nwg = (int)gridDim.x, orig = (int)blockIdx.x, xcd = orig % 8, q8 = nwg / 8, r8 = nwg % 8;
    const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int tm = bid / tiles_n, tn = bid % tiles_n;
    const int m0 = tm * BM, n0 = tn * GB_N;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    const uint16_t* srcA[IA];
    const uint16_t* srcB[IB];
#pragma unroll
    for (int i = 0; i < IA; ++i) {
        const int q = (i * NW + wave) * 64 + lane, row = q >> 3, pos = q & 7;
        srcA[i] = A + (size_t)(m0 + row) * K + 8 * (pos ^ (row & 7));
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
        const int q = (i * NW + wave) * 64 + lane, row = q >> 3, pos = q & 7;
        srcB[i] = W + (size_t)(n0 + row) * K + 8 * (pos ^ (row & 7));
    }
    auto stage = [&](int k0, int buf) {
        uint16_t* sA = smem + buf * (SA + SB);
        uint16_t* sB = sA + SA;
#pragma unroll
        for (int i = 0; i < IA; ++i)
            __builtin_amdgcn_global_load_lds((gptr_t)(srcA[i] + k0), (lptr_t)(sA + (i * NW + wave) * 512), 16, 0, 0);
#pragma unroll
        for (int i = 0; i < IB; ++i)
            __builtin_amdgcn_global_load_lds((gptr_t)(srcB[i] + k0), (lptr_t)(sB + (i * NW + wave) * 512), 16, 0, 0);
    };
    const int nk = K / GB_K;
    stage(0, 0);
    if (NB == 2) __syncthreads();                  // (its fence waits for the DMA: slab 0 is in LDS)
    float* sC = reinterpret_cast<float*>(smem);    // f32 [EG][128] epilogue image (after the loop)
    if (NB == 3) {
        // three slab buffers, two slabs in flight: slab k+2 is issued right after the barrier that
        // retires slab k, so the DMA spans a whole slab of MFMAs more; the barrier is a raw s_barrier
        // after a COUNTED vmcnt (a __syncthreads() fence would drain the DMA queue to 0,
        // cdna_hip_programming.md "Pipelining across barriers")
        static_assert(MF == 1, "three-buffer ring: 16x16x32 form only");
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
        const int r = lane & 15, h = lane >> 4;
        if (nk > 1) stage(GB_K, 1);
        int buf = 0, nbuf = 2;
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IA + IB) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of slab k-1 are done
            __builtin_amdgcn_s_barrier();
            if (kt + 2 < nk) stage((kt + 2) * GB_K, nbuf);         // into slab k-1's buffer
            const uint16_t* sA = smem + buf * (SA + SB);
            const uint16_t* sB = sA + SA;
#pragma unroll
            for (int ks = 0; ks < GB_K / 32; ++ks) {
                bf16x8 fa[4], fb[4];
                const int c = 4 * ks + h;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int ra = wm + 16 * i + r, rb = wn + 16 * i + r;
                    fa[i] = *reinterpret_cast<const bf16x8*>(sA + ra * GB_K + 8 * (c ^ (ra & 7)));
                    fb[i] = *reinterpret_cast<const bf16x8*>(sB + rb * GB_K + 8 * (c ^ (rb & 7)));
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
            buf = buf == 2 ? 0 : buf + 1;
            nbuf = nbuf == 2 ? 0 : nbuf + 1;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();              // every wave is done with the slabs: sC may overwrite them
#pragma unroll
        for (int g = 0; g < BM / EG; ++g) {
            if (wm >= EG * g && wm < EG * (g + 1)) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int reg = 0; reg < 4; ++reg)
                            sC[(wm - EG * g + 16 * i + 4 * h + reg) * GB_N + wn + 16 * j + r] = acc[i][j][reg];
            }
            gemm_finish<EPI, NT, EG>(sC, bias, R, C, m0 + EG * g, n0, N);
        }
    } else if (MF == 0) {
        // 2 x 2 v_mfma_f32_32x32x16_bf16 per 16-deep step
        f32x16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
        const int r = lane & 31, h = lane >> 5;
        for (int kt = 0; kt < nk; ++kt) {
            const int buf = kt & 1;
            if (kt + 1 < nk) stage((kt + 1) * GB_K, buf ^ 1);      // runs under this slab's MFMAs
            const uint16_t* sA = smem + buf * (SA + SB);
            const uint16_t* sB = sA + SA;
#pragma unroll
            for (int ks = 0; ks < GB_K / 16; ++ks) {
                bf16x8 fa[2], fb[2];
                const int c = 2 * ks + h;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int ra = wm + 32 * i + r, rb = wn + 32 * i + r;
                    fa[i] = *reinterpret_cast<const bf16x8*>(sA + ra * GB_K + 8 * (c ^ (ra & 7)));
                    fb[i] = *reinterpret_cast<const bf16x8*>(sB + rb * GB_K + 8 * (c ^ (rb & 7)));
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
            }
            __syncthreads();                       // slab k+1 landed (DMA retired); slab k's buffer is free
        }
#pragma unroll
        for (int g = 0; g < BM / EG; ++g) {
            if (wm >= EG * g && wm < EG * (g + 1)) {   // C/D map: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
#pragma unroll
                        for (int reg = 0; reg < 16; ++reg)
                            sC[(wm - EG * g + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h) * GB_N + wn + 32 * j + r] =
                                acc[i][j][reg];
            }
            gemm_finish<EPI, NT, EG>(sC, bias, R, C, m0 + EG * g, n0, N);
        }
    } else {
        // 4 x 4 v_mfma_f32_16x16x32_bf16 per 32-deep step (lane l: A[l & 15][8 (l >> 4) + j])
        f32x4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{};
        const int r = lane & 15, h = lane >> 4;
        for (int kt = 0; kt < nk; ++kt) {
            const int buf = kt & 1;
            if (kt + 1 < nk) stage((kt + 1) * GB_K, buf ^ 1);
            const uint16_t* sA = smem + buf * (SA + SB);
            const uint16_t* sB = sA + SA;
#pragma unroll
            for (int ks = 0; ks < GB_K / 32; ++ks) {
                bf16x8 fa[4], fb[4];
                const int c = 4 * ks + h;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int ra = wm + 16 * i + r, rb = wn + 16 * i + r;
                    fa[i] = *reinterpret_cast<const bf16x8*>(sA + ra * GB_K + 8 * (c ^ (ra & 7)));
                    fb[i] = *reinterpret_cast<const bf16x8*>(sB + rb * GB_K + 8 * (c ^ (rb & 7)));
                }
                if (GEMM_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
                if (GEMM_PRIO) __builtin_amdgcn_s_setprio(0);
            }
            __syncthreads();
        }
#pragma unroll
        for (int g = 0; g < BM / EG; ++g) {
            if (wm >= EG * g && wm < EG * (g + 1)) {   // C/D map: col = lane & 15, row = 4 (lane >> 4) + reg
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
#pragma unroll
                        for (int reg = 0; reg < 4; ++reg)
                            sC[(wm - EG * g + 16 * i + 4 * h + reg) * GB_N + wn + 16 * j + r] = acc[i][j][reg];
            }
            gemm_finish<EPI, NT, EG>(sC, bias, R, C, m0 + EG * g, n0, N);
        }
    }
    (void)M;
}

// wave-wide sum
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
    return v;
}

// one wavefront per row (H <= 64 * 16)
constexpr int LN_PER = 16;
__global__ __launch_bounds__(256) void k_layernorm(const uint16_t* __restrict__ x, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, uint16_t* __restrict__ y, int M,
                                                   int H, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    float v[LN_PER];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < LN_PER; ++k) {
        const int c = lane + 64 * k;
        v[k] = c < H ? bf2f(x[(size_t)row * H + c]) : 0.f;
        s += v[k];
    }
    const float mean = wave_sum(s) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < LN_PER; ++k) {
        const int c = lane + 64 * k;
        const float d = c < H ? v[k] - mean : 0.f;
        q += d * d;
    }
    const float inv = rsqrtf(wave_sum(q) / (float)H + eps);
#pragma unroll
    for (int k = 0; k < LN_PER; ++k) {
        const int c = lane + 64 * k;
        if (c < H) y[(size_t)row * H + c] = f2bf((v[k] - mean) * inv * gamma[c] + beta[c]);
    }
}

__global__ __launch_bounds__(256) void k_embed(const int32_t* __restrict__ ids, const uint16_t* __restrict__ wemb,
                                               const uint16_t* __restrict__ pemb, const uint16_t* __restrict__ temb,
                                               const float* __restrict__ gamma, const float* __restrict__ beta,
                                               uint16_t* __restrict__ out, int M, int S, int H, float eps) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    const int id = ids[row], pos = row % S;
    float v[LN_PER];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < LN_PER; ++k) {
        const int c = lane + 64 * k;
        v[k] = c < H ? bf2f(wemb[(size_t)id * H + c]) + bf2f(pemb[(size_t)pos * H + c]) + bf2f(temb[c]) : 0.f;
        s += v[k];
    }
    const float mean = wave_sum(s) / (float)H;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < LN_PER; ++k) {
        const int c = lane + 64 * k;
        const float d = c < H ? v[k] - mean : 0.f;
        q += d * d;
    }
    const float inv = rsqrtf(wave_sum(q) / (float)H + eps);
#pragma unroll
    for (int k = 0; k < LN_PER; ++k) {
        const int c = lane + 64 * k;
        if (c < H) out[(size_t)row * H + c] = f2bf((v[k] - mean) * inv * gamma[c] + beta[c]);
    }
}

// One workgroup per (sequence, head): K and V of the head staged in LDS as f32, one thread per query
// row with an online softmax (masked keys skipped, as HF's additive finfo.min mask makes them 0).
constexpr int ATT_D = 64, ATT_SMAX = 256;     // K and V of a head as f32 in LDS: 2 x 256 x 64 x 4 B
__global__ __launch_bounds__(256) void k_attention(const uint16_t* __restrict__ qkv, const int32_t* __restrict__ mask,
                                                   uint16_t* __restrict__ out, int S, int heads) {
    extern __shared__ float smem[];
    const int b = blockIdx.x / heads, hd = blockIdx.x % heads;
    const int H = heads * ATT_D, W3 = 3 * H;
    float* sK = smem;                        // [S][64]
    float* sV = smem + S * ATT_D;            // [S][64]
    int* sM = reinterpret_cast<int*>(sV + S * ATT_D);
    for (int i = threadIdx.x; i < S * ATT_D; i += blockDim.x) {
        const int j = i / ATT_D, d = i % ATT_D;
        const size_t base = (size_t)(b * S + j) * W3;
        sK[i] = bf2f(qkv[base + H + hd * ATT_D + d]);
        sV[i] = bf2f(qkv[base + 2 * H + hd * ATT_D + d]);
    }
    for (int j = threadIdx.x; j < S; j += blockDim.x) sM[j] = mask ? mask[b * S + j] : 1;
    __syncthreads();
    const float scale = 0.125f;              // 1 / sqrt(64)
    for (int qi = threadIdx.x; qi < S; qi += blockDim.x) {
        float q[ATT_D], o[ATT_D];
        const size_t qb = (size_t)(b * S + qi) * W3 + hd * ATT_D;
#pragma unroll
        for (int d = 0; d < ATT_D; ++d) {
            q[d] = bf2f(qkv[qb + d]) * scale;
            o[d] = 0.f;
        }
        float mx = -3.0e38f, l = 0.f;
        for (int j = 0; j < S; ++j) {
            if (!sM[j]) continue;
            const float* kr = sK + j * ATT_D;
            float sc = 0.f;
#pragma unroll
            for (int d = 0; d < ATT_D; ++d) sc += q[d] * kr[d];
            const float mn = fmaxf(mx, sc);
            const float a = __expf(mx - mn), p = __expf(sc - mn);
            l = l * a + p;
            const float* vr = sV + j * ATT_D;
#pragma unroll
            for (int d = 0; d < ATT_D; ++d) o[d] = o[d] * a + p * vr[d];
            mx = mn;
        }
        const float inv = l > 0.f ? 1.f / l : 0.f;
        const size_t ob = (size_t)(b * S + qi) * H + hd * ATT_D;
#pragma unroll
        for (int d = 0; d < ATT_D; ++d) out[ob + d] = f2bf(o[d] * inv);
    }
}

// Attention on the matrix cores, one workgroup (4 wavefronts) per (sequence, head), S <= 128 keys,
// S % 32 == 0.  Wavefront w owns queries [32w, 32w + 32).
//   X = K . Q^T  (32x32x16: A = K rows, B[d][query] = Q rows -- both K-contiguous)  -> X[key][query]:
//   per lane one query (its column), the keys in its 16 registers x 4 key tiles x the 2 lane halves,
//   so the softmax over keys is in-lane plus one shuffle across the halves.
//   Y = V^T . P  sums over X's ROW index, so P (= exp(X - max), bf16) is the B operand straight from
//   the accumulator registers (no lane movement); its k order inside a 16-step is permuted -- element
//   j of lane half h is key 16s + 8(j >> 2) + 4h + (j & 3) -- and the A operand (V^T, staged
//   transposed in LDS) is read in that same order.   O[query][d] = Y[d][query] / l[query].
constexpr int AT_ROW = ATT_D + 8;          // Q / K LDS rows: 64 bf16 + 16 B pad
constexpr int AT_VROW = 128 + 8;           // V^T LDS rows: 128 keys + 16 B pad
__global__ __launch_bounds__(256) void k_attention_mfma(const uint16_t* __restrict__ qkv, const int32_t* __restrict__ mask,
                                                        uint16_t* __restrict__ out, int S, int heads) {
    __shared__ __attribute__((aligned(16))) uint16_t sQ[128 * AT_ROW];
    __shared__ __attribute__((aligned(16))) uint16_t sK[128 * AT_ROW];
    __shared__ __attribute__((aligned(16))) uint16_t sVt[ATT_D * AT_VROW];
    __shared__ int sM[128];
    const int b = blockIdx.x / heads, hd = blockIdx.x % heads;
    const int H = heads * ATT_D, W3 = 3 * H;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // stage Q, K (row-major) and V^T; 16-byte chunks: row j = q >> 3, d = 8 (q & 7)
    for (int q = tid; q < S * 8; q += 256) {
        const int j = q >> 3, d = 8 * (q & 7);
        const uint16_t* src = qkv + (size_t)(b * S + j) * W3 + hd * ATT_D + d;
        *reinterpret_cast<uint4*>(sQ + j * AT_ROW + d) = *reinterpret_cast<const uint4*>(src);
        *reinterpret_cast<uint4*>(sK + j * AT_ROW + d) = *reinterpret_cast<const uint4*>(src + H);
        const uint4 v = *reinterpret_cast<const uint4*>(src + 2 * H);
        const uint32_t vw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sVt[(d + 2 * e) * AT_VROW + j] = (uint16_t)(vw[e] & 0xffffu);
            sVt[(d + 2 * e + 1) * AT_VROW + j] = (uint16_t)(vw[e] >> 16);
        }
    }
    for (int j = tid; j < 128; j += 256) sM[j] = (j < S) ? (mask ? mask[b * S + j] : 1) : 0;
    __syncthreads();
    const int q0 = 32 * wave;
    if (q0 >= S) return;
    const int r = lane & 31, h = lane >> 5;
    const int nkt = S / 32;
    f32x16 X[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) X[i] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < ATT_D / 16; ++ks) {
        const bf16x8 fq = *reinterpret_cast<const bf16x8*>(sQ + (q0 + r) * AT_ROW + 16 * ks + 8 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i < nkt) {
                const bf16x8 fk = *reinterpret_cast<const bf16x8*>(sK + (32 * i + r) * AT_ROW + 16 * ks + 8 * h);
                X[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fk, fq, X[i], 0, 0, 0);
            }
    }
    // softmax over keys for this lane's query (key of register g in tile i: 32i + (g&3) + 8(g>>2) + 4h)
    float mx = -3.0e38f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int key = 32 * i + (g & 3) + 8 * (g >> 2) + 4 * h;
            const float v = (i < nkt && sM[key]) ? X[i][g] * 0.125f : -3.0e38f;
            X[i][g] = v;
            mx = fmaxf(mx, v);
        }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const float p = X[i][g] > -1.0e38f ? __expf(X[i][g] - mx) : 0.f;
            X[i][g] = p;
            l += p;
        }
    l += __shfl_xor(l, 32);
    // Y[d][query] = sum_key V^T[d][key] P[key][query]
    f32x16 Y[2] = {f32x16{}, f32x16{}};
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < nkt) {
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                bf16x8 fp;
#pragma unroll
                for (int j = 0; j < 8; ++j) fp[j] = (__bf16)X[i][8 * s2 + j];
                const int kb = 32 * i + 16 * s2 + 4 * h;          // keys kb + {0..3} and kb + 8 + {0..3}
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const uint16_t* vr = sVt + (32 * t + r) * AT_VROW + kb;
                    const uint2 lo = *reinterpret_cast<const uint2*>(vr);
                    const uint2 hi = *reinterpret_cast<const uint2*>(vr + 8);
                    bf16x8 fv;
                    const uint32_t w4[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        fv[2 * e] = __builtin_bit_cast(__bf16, (uint16_t)(w4[e] & 0xffffu));
                        fv[2 * e + 1] = __builtin_bit_cast(__bf16, (uint16_t)(w4[e] >> 16));
                    }
                    Y[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fv, fp, Y[t], 0, 0, 0);
                }
            }
        }
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const size_t ob = (size_t)(b * S + q0 + r) * H + hd * ATT_D;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int g = 0; g < 16; ++g) out[ob + 32 * t + (g & 3) + 8 * (g >> 2) + 4 * h] = f2bf(Y[t][g] * inv);
}

// logits[m][c] = h[m] . Wc[c] + bc[c]   (one wavefront per row)
__global__ __launch_bounds__(256) void k_classify(const uint16_t* __restrict__ h, const uint16_t* __restrict__ Wc,
                                                  const float* __restrict__ bc, float* __restrict__ logits, int M,
                                                  int H, int L) {
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (row >= M) return;
    for (int c = 0; c < L; ++c) {
        float s = 0.f;
        for (int k = lane; k < H; k += 64) s += bf2f(h[(size_t)row * H + k]) * bf2f(Wc[(size_t)c * H + k]);
        s = wave_sum(s);
        if (lane == 0) logits[(size_t)row * L + c] = s + bc[c];
    }
}

// ------------------------------------------------------------------ detector front and back end
// ner.py HashTokenizer.encode on the device, one thread per row: tokens are maximal [A-Za-z0-9_]+
// runs or single bytes that are neither word bytes nor whitespace (Python bytes-regex \s = " \t\n
// \v\f\r"), ASCII lower-cased, id = 1000 + fnv1a64(token) % (vocab - 1000); a row is [CLS] tokens
// [SEP] [PAD]..., at most S ids.  Token byte ranges (row relative) go to tok_lo / tok_hi.
__device__ __forceinline__ bool ner_word(uint32_t c) {
    return (c - 48u < 10u) || ((c | 32u) - 97u < 26u) || c == 95u;
}
__device__ __forceinline__ bool ner_space(uint32_t c) { return c == 32u || (c - 9u < 5u); }

__global__ __launch_bounds__(256) void k_tokenize(const uint8_t* __restrict__ text, const uint64_t* __restrict__ offs,
                                                  int n_rows, int S, int vocab, int32_t* __restrict__ ids,
                                                  int32_t* __restrict__ mask, uint32_t* __restrict__ tok_lo,
                                                  uint32_t* __restrict__ tok_hi, int32_t* __restrict__ n_tok) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const uint64_t b = offs[r], len = offs[r + 1] - b;
    const uint8_t* t = text + b;
    const size_t o = (size_t)r * S;
    int k = 0;
    ids[o] = CLS_ID;
    tok_lo[o] = tok_hi[o] = 0;
    ++k;
    uint64_t i = 0;
    while (i < len && k < S - 1) {
        const uint32_t c = t[i];
        if (ner_space(c)) {
            ++i;
            continue;
        }
        uint64_t h = 0xcbf29ce484222325ull;
        const uint64_t s0 = i;
        if (ner_word(c)) {
            while (i < len && ner_word(t[i])) {
                const uint32_t x = t[i] - 65u < 26u ? t[i] + 32u : t[i];
                h = (h ^ x) * 0x100000001b3ull;
                ++i;
            }
        } else {
            h = (h ^ c) * 0x100000001b3ull;     // (not a letter: lower() leaves it)
            ++i;
        }
        ids[o + k] = 1000 + (int32_t)(h % (uint64_t)(vocab - 1000));
        tok_lo[o + k] = (uint32_t)s0;
        tok_hi[o + k] = (uint32_t)i;
        ++k;
    }
    ids[o + k] = SEP_ID;
    tok_lo[o + k] = tok_hi[o + k] = 0;
    ++k;
    n_tok[r] = k;
    for (int j = 0; j < S; ++j) mask[o + j] = j < k ? 1 : 0;
    for (int j = k; j < S; ++j) {
        ids[o + j] = PAD_ID;
        tok_lo[o + j] = tok_hi[o + j] = 0;
    }
}

// ner.py decode_spans on the device, one thread per row: argmax label per token (first maximum, as
// torch.argmax), BIO-merged into PERSON_NAME byte spans, written as the engine's external candidates
// (include/pii_engine.h pii_scan_redact_device_ext): ext[r * S + j], ext_n[r].
struct ExtSpan {      // = pii_span (16 B)
    uint32_t utt, start, end;
    uint16_t info_type;
    uint8_t likelihood, flags;
};
__global__ __launch_bounds__(256) void k_ner_spans(const float* __restrict__ logits, int L,
                                                   const uint32_t* __restrict__ tok_lo,
                                                   const uint32_t* __restrict__ tok_hi,
                                                   const int32_t* __restrict__ n_tok, int n_rows, int S,
                                                   int info_type, int likelihood, ExtSpan* __restrict__ ext,
                                                   uint32_t* __restrict__ ext_n) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_rows) return;
    const size_t o = (size_t)r * S;
    const int nt = n_tok[r];
    uint32_t n = 0;
    int cs = -1, ce = -1;
    auto flush = [&]() {
        if (cs >= 0) {
            ExtSpan x;
            x.utt = (uint32_t)r;
            x.start = (uint32_t)cs;
            x.end = (uint32_t)ce;
            x.info_type = (uint16_t)info_type;
            x.likelihood = (uint8_t)likelihood;
            x.flags = 0;
            ext[o + n++] = x;
        }
        cs = -1;
    };
    for (int j = 0; j < nt; ++j) {
        const float* lg = logits + (o + j) * L;
        int lab = 0;
        float best = lg[0];
        for (int c = 1; c < L; ++c)
            if (lg[c] > best) {
                best = lg[c];
                lab = c;
            }
        const int s = (int)tok_lo[o + j], e = (int)tok_hi[o + j];
        if (e <= s) {                      // [CLS] / [SEP]
            flush();
        } else if (lab == 1 || (lab == 2 && cs < 0)) {
            flush();
            cs = s;
            ce = e;
        } else if (lab == 2) {
            ce = e;
        } else {
            flush();
        }
    }
    flush();
    ext_n[r] = n;
}

}  // namespace

extern "C" {

int ner_tokenize(const uint8_t* text, const uint64_t* offs, int n_rows, int S, int vocab, int32_t* ids, int32_t* mask,
                 uint32_t* tok_lo, uint32_t* tok_hi, int32_t* n_tok, void* stream) {
    if (!text || !offs || !ids || !mask || !tok_lo || !tok_hi || !n_tok || n_rows <= 0 || S < 2 || vocab <= 1000)
        return -1;
    k_tokenize<<<(n_rows + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(text, offs, n_rows, S, vocab, ids,
                                                                                  mask, tok_lo, tok_hi, n_tok);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ner_spans(const float* logits, int L, const uint32_t* tok_lo, const uint32_t* tok_hi, const int32_t* n_tok,
              int n_rows, int S, int info_type, int likelihood, void* ext, uint32_t* ext_n, void* stream) {
    if (!logits || !tok_lo || !tok_hi || !n_tok || !ext || !ext_n || n_rows <= 0 || L < 3 || S < 2 ||
        likelihood < 1 || likelihood > 5 || info_type < 0 || info_type > 0xffff)
        return -1;
    k_ner_spans<<<(n_rows + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(
        logits, L, tok_lo, tok_hi, n_tok, n_rows, S, info_type, likelihood, static_cast<ExtSpan*>(ext), ext_n);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ner_gemm(const void* A, const void* W, const void* bias, const void* resid, void* C, int M, int N, int K,
             int epi, void* stream) {
    if (!A || !W || !C || M % GB_M || N % GB_N || K % GB_K || M <= 0 || epi < 0 || epi > 2 || (epi == 2 && !resid))
        return -1;
    const uint16_t *a = static_cast<const uint16_t*>(A), *w = static_cast<const uint16_t*>(W);
    const uint16_t* rs = static_cast<const uint16_t*>(resid);
    uint16_t* c = static_cast<uint16_t*>(C);
    const float* b = static_cast<const float*>(bias);
    hipStream_t st = static_cast<hipStream_t>(stream);
    // k_gemm2 (two slab buffers, two workgroups per CU) while the tile count is a few rounds of the
    // chip's workgroup slots; past that (the NER on the redaction path: M = 524288 tokens) the
    // single-buffer k_gemm's 3-4 workgroups per CU hide the DMA better (QKV 759 vs 647 TFLOP/s there,
    // 597 vs 634 at M = 8192; tools/gemm_ab.py, GEMM_M)
    const long tiles = (long)(M / GB_M) * (N / GB_N);
    if (GEMM_PIPE && tiles <= 16L * 256) {
        // 256-row tiles when they still give every CU at least two tiles, else 128-row tiles
        const bool big = GEMM_BIG && M % 256 == 0 && (M / 256) * (N / GB_N) >= 512;
        if (big) {
            auto kern = epi == EPI_GELU ? k_gemm2<EPI_GELU, 256, GEMM_MF, GEMM_NB> : epi == EPI_RESID ? k_gemm2<EPI_RESID, 256, GEMM_MF, GEMM_NB>
                                                                                     : k_gemm2<EPI_BIAS, 256, GEMM_MF, GEMM_NB>;
            kern<<<(M / 256) * (N / GB_N), 512, 0, st>>>(a, w, b, rs, c, M, N, K);
        } else {
            auto kern = epi == EPI_GELU ? k_gemm2<EPI_GELU, 128, GEMM_MF, GEMM_NB> : epi == EPI_RESID ? k_gemm2<EPI_RESID, 128, GEMM_MF, GEMM_NB>
                                                                                     : k_gemm2<EPI_BIAS, 128, GEMM_MF, GEMM_NB>;
            kern<<<(M / 128) * (N / GB_N), 256, 0, st>>>(a, w, b, rs, c, M, N, K);
        }
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    const int blocks = (M / GB_M) * (N / GB_N);
    auto kern = epi == EPI_GELU ? k_gemm<EPI_GELU> : epi == EPI_RESID ? k_gemm<EPI_RESID> : k_gemm<EPI_BIAS>;
    kern<<<blocks, G_THREADS, 0, st>>>(a, w, b, rs, c, M, N, K);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ner_layernorm(const void* x, const float* gamma, const float* beta, void* y, int M, int H, float eps,
                  void* stream) {
    if (!x || !gamma || !beta || !y || H > 64 * LN_PER || M <= 0) return -1;
    k_layernorm<<<(M + 3) / 4, 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t*>(x), gamma, beta, static_cast<uint16_t*>(y), M, H, eps);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ner_embed(const int32_t* ids, const void* wemb, const void* pemb, const void* temb, const float* gamma,
              const float* beta, void* out, int M, int S, int H, float eps, void* stream) {
    if (!ids || !wemb || !pemb || !temb || !out || H > 64 * LN_PER || M <= 0 || S <= 0) return -1;
    k_embed<<<(M + 3) / 4, 256, 0, static_cast<hipStream_t>(stream)>>>(
        ids, static_cast<const uint16_t*>(wemb), static_cast<const uint16_t*>(pemb),
        static_cast<const uint16_t*>(temb), gamma, beta, static_cast<uint16_t*>(out), M, S, H, eps);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ner_attention(const void* qkv, const int32_t* mask, void* out, int B, int S, int heads, int dhead, void* stream) {
    if (!qkv || !out || dhead != ATT_D || S <= 0 || S > ATT_SMAX || B <= 0 || heads <= 0) return -1;
    if (S <= 128 && S % 32 == 0) {          // matrix-core path
        k_attention_mfma<<<B * heads, 256, 0, static_cast<hipStream_t>(stream)>>>(
            static_cast<const uint16_t*>(qkv), mask, static_cast<uint16_t*>(out), S, heads);
        return hipGetLastError() == hipSuccess ? 0 : -3;
    }
    const size_t lds = (size_t)S * ATT_D * 2 * sizeof(float) + (size_t)S * sizeof(int);
    static bool raised = false;
    if (lds > 64 * 1024 && !raised) {
        if (hipFuncSetAttribute((const void*)k_attention, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess)
            return -3;
        raised = true;
    }
    k_attention<<<B * heads, 256, lds, static_cast<hipStream_t>(stream)>>>(static_cast<const uint16_t*>(qkv), mask,
                                                                         static_cast<uint16_t*>(out), S, heads);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ner_classify(const void* h, const void* Wc, const float* bc, float* logits, int M, int H, int L, void* stream) {
    if (!h || !Wc || !bc || !logits || M <= 0 || L <= 0) return -1;
    k_classify<<<(M + 3) / 4, 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t*>(h), static_cast<const uint16_t*>(Wc), bc, logits, M, H, L);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // extern "C"

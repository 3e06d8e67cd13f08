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
// 64x64 quarter as 2x2 v_mfma_f32_32x32x16_bf16 tiles, K staged through LDS in 32-wide slabs (rows
// padded by 16 B so the 16-byte fragment reads hit 32 distinct banks), the next slab's global loads
// in flight while the current one is multiplied.  Operands are K-contiguous (activations row-major,
// nn.Linear weights [out, in]), which is exactly the MFMA's A / B lane map: lane l holds
// A[row l&31][k 8(l>>5) .. +7] and W[col l&31][same k] -- no transposes anywhere.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {      // round to nearest even (NaN kept quiet)
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

constexpr int GB_M = 128, GB_N = 128, GB_K = 32;
constexpr int G_THREADS = 256;
constexpr int LDS_ROW = GB_K + 8;      // bf16 per LDS row (64 B of data + 16 B pad)

enum { EPI_BIAS = 0, EPI_GELU = 1, EPI_RESID = 2 };

// C = A . W^T + bias (+ epilogue).  A [M, K], W [N, K], C / R [M, N] bf16; bias f32 [N].
// Requires M % 128 == 0, N % 128 == 0, K % 32 == 0 (the host pads M).
__global__ __launch_bounds__(G_THREADS) void k_gemm(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
                                                    const float* __restrict__ bias, const uint16_t* __restrict__ R,
                                                    uint16_t* __restrict__ C, int M, int N, int K, int epi) {
    __shared__ __attribute__((aligned(16))) uint16_t sA[2][GB_M * LDS_ROW];
    __shared__ __attribute__((aligned(16))) uint16_t sB[2][GB_N * LDS_ROW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-aware tile order: workgroups are dealt to the 8 XCDs round robin (id % 8), so renumber them
    // such that each XCD gets a contiguous run of tiles -- the N tiles of the same M row-block -- and
    // the A rows they share stay in that XCD's L2
    const int tiles_n = N / GB_N;
    const int nb = (int)gridDim.x;
    const int bid = nb % 8 == 0 ? (int)(blockIdx.x % 8) * (nb / 8) + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    const int tm = bid / tiles_n, tn = bid % tiles_n;
    const int m0 = tm * GB_M, n0 = tn * GB_N;
    const int wm = (wave >> 1) * 64, wn = (wave & 1) * 64;
    // global -> register staging: each thread moves 2 16-byte chunks of A and 2 of W per K slab
    // (128 rows x 64 B = 512 chunks per operand); chunk q: row q >> 2, 16-byte column q & 3
    uint4 ra[2], rb[2];
    auto gload = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = tid + i * G_THREADS, row = q >> 2, col = (q & 3) * 8;
            ra[i] = *reinterpret_cast<const uint4*>(A + (size_t)(m0 + row) * K + k0 + col);
            rb[i] = *reinterpret_cast<const uint4*>(W + (size_t)(n0 + row) * K + k0 + col);
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = tid + i * G_THREADS, row = q >> 2, col = (q & 3) * 8;
            *reinterpret_cast<uint4*>(&sA[buf][row * LDS_ROW + col]) = ra[i];
            *reinterpret_cast<uint4*>(&sB[buf][row * LDS_ROW + col]) = rb[i];
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};
    const int r = lane & 31, h = lane >> 5;
    const int nk = K / GB_K;
    gload(0);
    lstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) gload((kt + 1) * GB_K);          // next slab in flight during the MFMAs
#pragma unroll
        for (int ks = 0; ks < GB_K / 16; ++ks) {
            bf16x8 fa[2], fb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                fa[i] = *reinterpret_cast<const bf16x8*>(&sA[buf][(wm + 32 * i + r) * LDS_ROW + ks * 16 + 8 * h]);
                fb[i] = *reinterpret_cast<const bf16x8*>(&sB[buf][(wn + 32 * i + r) * LDS_ROW + ks * 16 + 8 * h]);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) lstore(buf ^ 1);
        __syncthreads();
    }
    // epilogue: C/D map of 32x32x16: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = n0 + wn + 32 * j + r;
            const float b = bias ? bias[col] : 0.f;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = m0 + wm + 32 * i + (reg & 3) + 8 * (reg >> 2) + 4 * h;
                float v = acc[i][j][reg] + b;
                if (epi == EPI_GELU) v = 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
                else if (epi == EPI_RESID) v += bf2f(R[(size_t)row * N + col]);
                C[(size_t)row * N + col] = f2bf(v);
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

}  // namespace

extern "C" {

int ner_gemm(const void* A, const void* W, const void* bias, const void* resid, void* C, int M, int N, int K,
             int epi, void* stream) {
    if (!A || !W || !C || M % GB_M || N % GB_N || K % GB_K || M <= 0 || epi < 0 || epi > 2 || (epi == 2 && !resid))
        return -1;
    const int blocks = (M / GB_M) * (N / GB_N);
    k_gemm<<<blocks, G_THREADS, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(W), static_cast<const float*>(bias),
        static_cast<const uint16_t*>(resid), static_cast<uint16_t*>(C), M, N, K, epi);
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

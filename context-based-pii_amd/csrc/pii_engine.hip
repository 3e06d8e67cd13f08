// pii_engine.hip - MI355X (gfx950) scan-and-redact engine: kernels + C ABI (include/pii_engine.h).
//
// Replaces the remote de-identification call of the reference,
//   main_service/main.py:728  dlp_client.deidentify_content(request)   (inside call_dlp_for_redaction,
//   main.py:580-773), and the Redis context record main.py:366-374 / 403.
//
// Pipeline per batch (one HIP stream, no host round trip until pii_sync):
//   k_chunk_index  lane -> utterance ranges of ~BYTES_PER_LANE bytes (load balance, no halo needed)
//   k_scan         REVERSE two-automaton DFA scan, tables in LDS.  D = relaxed detector prefilter,
//                  K = exact context keywords.  Emits candidate STARTS (events) per utterance and the
//                  agent-row context group (extract_expected_pii, main.py:558-578)
//   k_ctx_scan / k_ctx_apply   per-conversation context (Redis SETEX/GET + TTL) as a segmented scan
//   k_resolve      per utterance: leftmost-first confirmation (FIRST DFAs), validators, hotword
//                  windows (HOT DFAs), exclusion, overlap resolution, output sizing
//   k_scan_*       exclusive scans -> output byte offsets and span offsets
//   k_finalize     capacity / error check (device side)
//   k_redact       prefix-sum scatter of kept bytes and "[INFO_TYPE]" tokens, span list, histogram
//   k_ctx_commit   write the per-conversation context back (only when the call succeeded)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pii_engine.h"
#include "pii_device.h"

using namespace pii;

namespace {

constexpr int P_MAX = 64;          // detector patterns handled by k_resolve's private state
constexpr int NE_MAX = 8;          // excluder patterns
constexpr int SCAN_BLOCK = 512;
constexpr int CTX_BLOCK = 1024;
constexpr int SCAN_ITEMS = 4;      // items per thread in the offset scans
constexpr int SCAN_TILE = 256 * SCAN_ITEMS;
constexpr uint32_t BYTES_PER_LANE = 2048;
constexpr int KW_NONE = 0x7fff;

enum : uint32_t { ERR_CAPACITY = 1, ERR_ORDER = 2, ERR_SLOT = 4 };

struct Event {
    uint32_t pos;   // candidate start, relative to the utterance
    uint32_t acc;   // SCAN-D accept-set id of the transition that reported it
};

struct RulesDev {
    int P, G, T, V, SD, CD, d_start, SK, CK, k_start, n_hot, min_len;
    int kw_always_min, NE;
    const uint16_t* cmap2;    // [256] classD | classK << 8
    const uint16_t* td;       // [SD*CD] premultiplied next row | 0x8000 accept
    const uint16_t* tk;       // [SK*CK]
    const uint16_t* d_accid;  // [SD*CD]
    const uint32_t* d_acc_off;
    const uint16_t* d_acc_ids;
    const uint16_t* k_accid;  // [SK*CK]
    const uint16_t* k_acc_min;  // per K accept set: smallest context group
    const uint16_t* det_type;
    const uint8_t* det_val;
    const uint8_t* det_lik;
    const uint8_t* det_exidx;   // excluder slot or 0xff
    const int32_t* first_desc;  // [P*8]
    const int32_t* hot_rule;    // [n_hot*4] wb, wa, fixed, rel
    const int32_t* hot_desc;    // [n_hot*8]
    Pool pool;
    const uint8_t* var_enabled;  // [V*T]
    const uint8_t* var_minlik;   // [V]
    const uint32_t* rule_off;    // [V*T+1]
    const uint16_t* rule_ids;
    const uint32_t* excl_off;    // [V*T+1]
    const uint16_t* excl_ids;
    const uint32_t* tok_off;     // [T+1] into tok_bytes: "[NAME]"
    const uint8_t* tok_bytes;
};

// ------------------------------------------------------------------------------- k_chunk_index
__global__ void k_chunk_index(const uint64_t* __restrict__ offs, uint32_t n_utt, uint32_t n_chunks,
                              uint32_t* __restrict__ first_utt) {
    uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u > n_utt) return;
    const uint64_t base = offs[0];
    const uint64_t su = offs[u] - base;
    uint64_t c_lo = 0;
    if (u > 0) c_lo = (offs[u - 1] - base) / BYTES_PER_LANE + 1;
    uint64_t c_hi = (u == n_utt) ? n_chunks : su / BYTES_PER_LANE;
    if (c_hi > n_chunks) c_hi = n_chunks;
    for (uint64_t c = c_lo; c <= c_hi; ++c) first_utt[c] = u;
}

// ------------------------------------------------------------------------------------- k_scan
__device__ __forceinline__ uint32_t byte_of(const uint4& w, int k) {
    uint32_t x = (k & 8) ? ((k & 4) ? w.w : w.z) : ((k & 4) ? w.y : w.x);
    return (x >> ((k & 3) * 8)) & 0xffu;
}

template <int K>
__device__ __forceinline__ uint32_t byte_c(const uint4& w) {
    const uint32_t x = (K & 8) ? ((K & 4) ? w.w : w.z) : ((K & 4) ? w.y : w.x);
    return (x >> ((K & 3) * 8)) & 0xffu;
}

struct ScanLane {
    uint32_t sd, sk, cnt, kmask;
    int kwmin;
    Event* evu;
    int64_t s;
};

__device__ __forceinline__ void scan_step(const RulesDev& R, const uint16_t* s_cmap, const uint16_t* s_td,
                                          const uint16_t* s_tk, ScanLane& L, uint32_t b, int64_t j) {
    const uint32_t cc = s_cmap[b];
    const uint32_t nd = s_td[L.sd + (cc & 0xffu)];
    const uint32_t nk = s_tk[L.sk + (cc >> 8)];
    if (__builtin_expect(((nd | (nk & L.kmask)) & 0x8000u) != 0, 0)) {
        if (nd & 0x8000u) {
            Event e;
            e.pos = (uint32_t)(j + 1 - L.s);
            e.acc = R.d_accid[L.sd + (cc & 0xffu)];
            L.evu[L.cnt++] = e;
        }
        if (nk & L.kmask & 0x8000u) {
            const int g = R.k_acc_min[R.k_accid[L.sk + (cc >> 8)]];
            L.kwmin = g < L.kwmin ? g : L.kwmin;
        }
    }
    L.sd = nd & 0x7fffu;
    L.sk = nk & 0x7fffu;
}

__global__ __launch_bounds__(SCAN_BLOCK) void k_scan(const RulesDev R, const uint8_t* __restrict__ text,
                                                     const uint64_t* __restrict__ offs, uint32_t n_utt,
                                                     const uint8_t* __restrict__ role,
                                                     const uint32_t* __restrict__ first_utt, uint32_t n_chunks,
                                                     Event* __restrict__ ev, uint32_t* __restrict__ n_ev,
                                                     int16_t* __restrict__ kw_group) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem32[];
    uint16_t* s_cmap = reinterpret_cast<uint16_t*>(smem32);
    const int nd_words = (R.SD * R.CD + 1) / 2;
    const int nk_words = (R.SK * R.CK + 1) / 2;
    uint16_t* s_td = s_cmap + 256;
    uint16_t* s_tk = s_td + nd_words * 2;
    {
        const uint32_t* g_cmap = reinterpret_cast<const uint32_t*>(R.cmap2);
        const uint32_t* g_td = reinterpret_cast<const uint32_t*>(R.td);
        const uint32_t* g_tk = reinterpret_cast<const uint32_t*>(R.tk);
        uint32_t* d_td = smem32 + 128;
        uint32_t* d_tk = d_td + nd_words;
        for (int i = threadIdx.x; i < 128; i += blockDim.x) smem32[i] = g_cmap[i];
        for (int i = threadIdx.x; i < nd_words; i += blockDim.x) d_td[i] = g_td[i];
        for (int i = threadIdx.x; i < nk_words; i += blockDim.x) d_tk[i] = g_tk[i];
    }
    __syncthreads();
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    const uint64_t base = offs[0];
    const uint64_t total_end = offs[n_utt];
    const uintptr_t lo_ok = (uintptr_t)(text + base);
    const uintptr_t hi_ok = (uintptr_t)(text + total_end);
    const uint32_t u1 = first_utt[c + 1];
    for (uint32_t u = first_utt[c]; u < u1; ++u) {
        const int64_t s = (int64_t)offs[u];
        const int64_t e = (int64_t)offs[u + 1];
        const bool agent = role[u] == PII_ROLE_AGENT;
        ScanLane L;
        L.sd = (uint32_t)R.d_start;
        L.sk = (uint32_t)R.k_start;
        L.cnt = 0;
        L.kmask = agent ? 0xffffu : 0u;
        L.kwmin = R.kw_always_min;
        L.evu = ev + (s - (int64_t)base);
        L.s = s;
        int64_t j = e - 1;
        while (j >= s) {
            const uintptr_t a = (uintptr_t)(text + j);
            const uintptr_t cb = a & ~(uintptr_t)15;
            const int k_hi = (int)(a & 15);
            const int64_t room = j - s;
            const int k_lo = room >= k_hi ? 0 : k_hi - (int)room;
            if (cb >= lo_ok && cb + 16 <= hi_ok) {
                const uint4 w = *reinterpret_cast<const uint4*>(cb);
                if (k_hi == 15 && k_lo == 0) {
                    const int64_t j0 = j - 15;
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<15>(w), j0 + 15);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<14>(w), j0 + 14);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<13>(w), j0 + 13);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<12>(w), j0 + 12);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<11>(w), j0 + 11);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<10>(w), j0 + 10);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<9>(w), j0 + 9);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<8>(w), j0 + 8);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<7>(w), j0 + 7);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<6>(w), j0 + 6);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<5>(w), j0 + 5);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<4>(w), j0 + 4);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<3>(w), j0 + 3);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<2>(w), j0 + 2);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<1>(w), j0 + 1);
                    scan_step(R, s_cmap, s_td, s_tk, L, byte_c<0>(w), j0 + 0);
                } else {
                    for (int k = k_hi; k >= k_lo; --k) scan_step(R, s_cmap, s_td, s_tk, L, byte_of(w, k), j - (k_hi - k));
                }
            } else {
                for (int k = k_hi; k >= k_lo; --k) {
                    const int64_t jj = j - (k_hi - k);
                    scan_step(R, s_cmap, s_td, s_tk, L, text[jj], jj);
                }
            }
            j -= (k_hi - k_lo + 1);
        }
        // beginning of the utterance: the end-of-text pseudo class of the reverse automata
        {
            const uint32_t nd = s_td[L.sd + (uint32_t)(R.CD - 1)];
            const uint32_t nk = s_tk[L.sk + (uint32_t)(R.CK - 1)];
            if (nd & 0x8000u) {
                Event evt;
                evt.pos = 0;
                evt.acc = R.d_accid[L.sd + (uint32_t)(R.CD - 1)];
                L.evu[L.cnt++] = evt;
            }
            if (nk & L.kmask & 0x8000u) {
                const int g = R.k_acc_min[R.k_accid[L.sk + (uint32_t)(R.CK - 1)]];
                L.kwmin = g < L.kwmin ? g : L.kwmin;
            }
        }
        n_ev[u] = L.cnt;
        kw_group[u] = (int16_t)((agent && L.kwmin != KW_NONE) ? L.kwmin : -1);
    }
}

// ---------------------------------------------------------------------------- context (a11)
// segmented (by conversation run) scan of "latest agent row with a context hit"
struct SegV {
    uint32_t f;
    int32_t v;
};
__device__ __forceinline__ SegV seg_combine(SegV a, SegV b) {
    SegV r;
    r.f = a.f | b.f;
    r.v = b.f ? b.v : (a.v > b.v ? a.v : b.v);
    return r;
}

__global__ __launch_bounds__(CTX_BLOCK) void k_ctx_scan(const uint32_t* __restrict__ slot, const uint8_t* __restrict__ role,
                                                        const int16_t* __restrict__ kw, uint32_t n_utt, uint32_t n_slots,
                                                        uint32_t* __restrict__ incl, int32_t* __restrict__ agg_v,
                                                        uint32_t* __restrict__ agg_f, uint32_t* __restrict__ stamp,
                                                        uint32_t epoch, uint32_t* __restrict__ err) {
    __shared__ SegV wsum[CTX_BLOCK / 64];
    const uint32_t u = blockIdx.x * CTX_BLOCK + threadIdx.x;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    SegV x;
    x.f = 0;
    x.v = -1;
    if (u < n_utt) {
        const uint32_t sl = slot[u];
        if (sl >= n_slots) atomicOr(err, (uint32_t)ERR_SLOT);
        const bool start = (u == 0) || slot[u - 1] != sl;
        x.f = start ? 1u : 0u;
        x.v = (role[u] == PII_ROLE_AGENT && kw[u] >= 0) ? (int32_t)u : -1;
        if (start && sl < n_slots) {
            const uint32_t old = atomicExch(&stamp[sl], epoch);
            if (old == epoch) atomicOr(err, (uint32_t)ERR_ORDER);
        }
    }
    for (int d = 1; d < 64; d <<= 1) {
        SegV o;
        o.f = __shfl_up(x.f, d);
        o.v = __shfl_up(x.v, d);
        if (lane >= d) x = seg_combine(o, x);
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < CTX_BLOCK / 64; ++w) wsum[w] = seg_combine(wsum[w - 1], wsum[w]);
    }
    __syncthreads();
    if (wid > 0) x = seg_combine(wsum[wid - 1], x);
    if (u < n_utt) incl[u] = (x.f ? 0x80000000u : 0u) | (uint32_t)(x.v + 1);
    if (threadIdx.x == CTX_BLOCK - 1 || u == n_utt - 1) {
        agg_v[blockIdx.x] = x.v;
        agg_f[blockIdx.x] = x.f;
    }
}

__device__ __forceinline__ int32_t ctx_carry(const int32_t* agg_v, const uint32_t* agg_f, int64_t blk) {
    for (int64_t b = blk - 1; b >= 0; --b) {
        if (agg_v[b] >= 0) return agg_v[b];
        if (agg_f[b]) return -1;
    }
    return -1;
}

__global__ void k_ctx_apply(const uint32_t* __restrict__ slot, const uint8_t* __restrict__ role,
                            const int16_t* __restrict__ kw, const int64_t* __restrict__ ts, uint32_t n_utt,
                            uint32_t n_slots, int64_t ttl_us, const uint32_t* __restrict__ incl,
                            const int32_t* __restrict__ agg_v, const uint32_t* __restrict__ agg_f,
                            const int32_t* __restrict__ st_group, const int64_t* __restrict__ st_ts,
                            int16_t* __restrict__ ctx, int32_t* __restrict__ commit) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_utt) return;
    const uint32_t sl = slot[u];
    const int64_t blk = u / CTX_BLOCK;
    const bool start = (u == 0) || slot[u - 1] != sl;
    // hit strictly before u in the same run
    int32_t prev = -1;
    if (!start) {
        const uint32_t pv = incl[u - 1];
        const bool same_blk = (u % CTX_BLOCK) != 0;
        prev = same_blk ? (int32_t)(pv & 0x7fffffffu) - 1 : -1;
        const bool run_started_in_blk = same_blk && (pv & 0x80000000u);
        if (prev < 0 && !run_started_in_blk) prev = ctx_carry(agg_v, agg_f, blk);
    }
    const uint8_t r = role[u];
    int16_t used = -1;
    if (r == PII_ROLE_CUSTOMER && sl < n_slots) {
        int32_t g;
        int64_t t;
        if (prev >= 0) {
            g = kw[prev];
            t = ts ? ts[prev] : 0;
        } else {
            g = st_group[sl];
            t = st_ts[sl];
        }
        const int64_t now = ts ? ts[u] : 0;
        if (g >= 0 && (ts == nullptr || now - t < ttl_us)) used = (int16_t)g;
    }
    ctx[u] = (r == PII_ROLE_AGENT) ? kw[u] : used;
    // last row of the run: the latest hit of the whole run (to be committed)
    const bool last = (u == n_utt - 1) || slot[u + 1] != sl;
    if (last) {
        int32_t full = (r == PII_ROLE_AGENT && kw[u] >= 0) ? (int32_t)u : prev;
        commit[u] = full;
    }
}

__global__ void k_ctx_commit(const uint32_t* __restrict__ slot, const int16_t* __restrict__ kw,
                             const int64_t* __restrict__ ts, uint32_t n_utt, uint32_t n_slots,
                             const int32_t* __restrict__ commit, const uint32_t* __restrict__ err,
                             int32_t* __restrict__ st_group, int64_t* __restrict__ st_ts) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_utt || *err != 0) return;
    const uint32_t sl = slot[u];
    const bool last = (u == n_utt - 1) || slot[u + 1] != sl;
    if (!last || sl >= n_slots) return;
    const int32_t j = commit[u];
    if (j >= 0) {
        st_group[sl] = kw[j];
        st_ts[sl] = ts ? ts[j] : 0;
    }
}

// ---------------------------------------------------------------------------------- k_resolve
__global__ __launch_bounds__(256) void k_resolve(const RulesDev R, const uint8_t* __restrict__ text,
                                                 const uint64_t* __restrict__ offs, uint32_t n_utt,
                                                 const uint8_t* __restrict__ role, const int16_t* __restrict__ ctx,
                                                 const Event* __restrict__ ev, const uint32_t* __restrict__ n_ev,
                                                 pii_span* __restrict__ fd, uint32_t* __restrict__ n_find,
                                                 uint32_t* __restrict__ out_len) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= n_utt) return;
    const uint64_t base = offs[0];
    const uint64_t s_abs = offs[u], e_abs = offs[u + 1];
    const int L = (int)(e_abs - s_abs);
    const uint8_t* t0 = text + s_abs;
    const uint32_t ne = n_ev[u];
    const Event* evu = ev + (s_abs - base);
    pii_span* fdu = fd + (s_abs - base) / (uint64_t)R.min_len;
    const int v = (role[u] == PII_ROLE_CUSTOMER && ctx[u] >= 0) ? ctx[u] + 1 : 0;
    const int T = R.T;
    const int minlik = R.var_minlik[v];
    uint32_t cur[P_MAX];
    uint64_t touched = 0;
    int ex_s[NE_MAX], ex_e[NE_MAX], ex_t[NE_MAX];
    uint32_t ex_valid = 0;
    int max_end = 0;
    uint32_t nf = 0;
    int64_t out = L;
    for (int k = (int)ne - 1; k >= 0; --k) {
        const Event E = evu[k];
        const int s = (int)E.pos;
        const uint32_t a0 = R.d_acc_off[E.acc], a1 = R.d_acc_off[E.acc + 1];
        int best_e = -1, best_t = 0, best_lik = 0;
        for (uint32_t i = a0; i < a1; ++i) {
            const int p = R.d_acc_ids[i];
            const int t = R.det_type[p];
            if (!R.var_enabled[v * T + t]) continue;
            if (((touched >> p) & 1) && (uint32_t)s < cur[p]) continue;
            const int e = first_run(R.pool, R.first_desc + 8 * p, t0, s, L);
            if (e < 0) continue;
            cur[p] = (uint32_t)e;
            touched |= 1ull << p;
            const int xi = R.det_exidx[p];
            if (!validate(R.det_val[p], t0 + s, e - s)) {
                if (xi != 0xff) ex_valid &= ~(1u << xi);
                continue;
            }
            int lik = R.det_lik[p];
            const uint32_t r0 = R.rule_off[v * T + t], r1 = R.rule_off[v * T + t + 1];
            for (uint32_t q = r0; q < r1; ++q) {
                const int h = R.rule_ids[q];
                const int wb = R.hot_rule[4 * h], wa = R.hot_rule[4 * h + 1];
                const int fixed = R.hot_rule[4 * h + 2], rel = R.hot_rule[4 * h + 3];
                bool hit = false;
                if (wb > 0) hit = hot_run(R.pool, R.hot_desc + 8 * h, t0, s - wb > 0 ? s - wb : 0, s);
                if (!hit && wa > 0) hit = hot_run(R.pool, R.hot_desc + 8 * h, t0, e, e + wa < L ? e + wa : L);
                if (hit) {
                    if (fixed) lik = fixed;
                    else {
                        lik += rel;
                        lik = lik < 1 ? 1 : (lik > 5 ? 5 : lik);
                    }
                }
            }
            if (lik < minlik) {
                if (xi != 0xff) ex_valid &= ~(1u << xi);
                continue;
            }
            if (xi != 0xff) {
                ex_s[xi] = s;
                ex_e[xi] = e;
                ex_t[xi] = t;
                ex_valid |= 1u << xi;
            }
            // exclusion (FULL_MATCH): inside a finding of an excluded type (A.5)
            const uint32_t x0 = R.excl_off[v * T + t], x1 = R.excl_off[v * T + t + 1];
            bool excluded = false;
            for (uint32_t q = x0; q < x1 && !excluded; ++q) {
                const int xt = R.excl_ids[q];
                for (int x = 0; x < R.NE; ++x) {
                    if (x == xi || !((ex_valid >> x) & 1) || ex_t[x] != xt) continue;
                    if (ex_s[x] <= s && e <= ex_e[x]) {
                        excluded = true;
                        break;
                    }
                }
            }
            if (excluded) continue;
            // best at this start: longest, then most likely, then lowest type index (A.6)
            const bool better = best_e < 0 || e > best_e || (e == best_e && (lik > best_lik || (lik == best_lik && t < best_t)));
            if (better) {
                best_e = e;
                best_t = t;
                best_lik = lik;
            }
        }
        if (best_e >= 0 && s >= max_end) {
            pii_span f;
            f.utt = u;
            f.start = (uint32_t)s;
            f.end = (uint32_t)best_e;
            f.info_type = (uint16_t)best_t;
            f.likelihood = (uint8_t)best_lik;
            f.flags = 0;
            fdu[nf++] = f;
            max_end = best_e;
            out += (int64_t)(R.tok_off[best_t + 1] - R.tok_off[best_t]) - (best_e - s);
        }
    }
    n_find[u] = nf;
    out_len[u] = (uint32_t)out;
}

// ---------------------------------------------------------------------------- exclusive scans
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, int lane) {
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(x, d);
        if (lane >= d) x += o;
    }
    return x;
}

// block-level exclusive scan of 256 threads x SCAN_ITEMS; returns block total
__device__ uint64_t block_exscan(uint64_t (&v)[SCAN_ITEMS], uint64_t* sh) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t tsum = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint64_t x = v[i];
        v[i] = tsum;
        tsum += x;
    }
    const uint64_t inc = wave_incl_scan(tsum, lane);
    if (lane == 63) sh[wid] = inc;
    __syncthreads();
    uint64_t wpre = 0, total = 0;
    for (int w = 0; w < 4; ++w) {
        if (w < wid) wpre += sh[w];
        total += sh[w];
    }
    const uint64_t tpre = wpre + inc - tsum;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) v[i] += tpre;
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t* __restrict__ in, uint32_t n,
                                                     uint64_t* __restrict__ bsum) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t s = 0;
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint64_t idx = base + (uint64_t)i * 256 + threadIdx.x;
        if (idx < n) s += in[idx];
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    s = wave_incl_scan(s, lane);
    if (lane == 63) sh[wid] = s;
    __syncthreads();
    if (threadIdx.x == 0) bsum[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// single block: exclusive scan of nb block sums in place (serial over 256-thread chunks)
__global__ __launch_bounds__(256) void k_scan_blocks(uint64_t* __restrict__ bsum, uint32_t nb) {
    __shared__ uint64_t sh[4];
    uint64_t carry = 0;
    for (uint32_t c0 = 0; c0 < nb; c0 += SCAN_TILE) {
        uint64_t v[SCAN_ITEMS];
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const uint32_t idx = c0 + threadIdx.x * SCAN_ITEMS + i;
            v[i] = idx < nb ? bsum[idx] : 0;
        }
        const uint64_t tot = block_exscan(v, sh);
        for (int i = 0; i < SCAN_ITEMS; ++i) {
            const uint32_t idx = c0 + threadIdx.x * SCAN_ITEMS + i;
            if (idx < nb) bsum[idx] = v[i] + carry;
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) bsum[nb] = carry;
}

// out[i] = exclusive prefix of in[]; out[n] = total
__global__ __launch_bounds__(256) void k_scan_apply(const uint32_t* __restrict__ in, uint32_t n,
                                                    const uint64_t* __restrict__ bsum, uint64_t* __restrict__ out) {
    __shared__ uint64_t sh[4];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE;
    uint64_t v[SCAN_ITEMS];
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint64_t idx = base + threadIdx.x * SCAN_ITEMS + i;
        v[i] = idx < n ? in[idx] : 0;
    }
    block_exscan(v, sh);
    const uint64_t off = bsum[blockIdx.x];
    for (int i = 0; i < SCAN_ITEMS; ++i) {
        const uint64_t idx = base + threadIdx.x * SCAN_ITEMS + i;
        if (idx < n) out[idx] = v[i] + off;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = bsum[gridDim.x];
}

__global__ void k_finalize(const uint64_t* __restrict__ out_offs, const uint64_t* __restrict__ span_offs,
                           uint32_t n_utt, uint64_t out_cap, uint64_t span_cap, uint32_t* __restrict__ err,
                           uint64_t* __restrict__ totals) {
    const uint64_t ob = out_offs[n_utt], ns = span_offs[n_utt];
    if (ob > out_cap || ns > span_cap) atomicOr(err, (uint32_t)ERR_CAPACITY);
    totals[0] = ob;
    totals[1] = ns;
    totals[2] = *err;
}

// ---------------------------------------------------------------------------------- k_redact
// one wavefront per utterance: copy kept byte runs and "[INFO_TYPE]" tokens to the prefix-summed
// output position; emit spans; per-type histogram through LDS.
constexpr int REDACT_BLOCK = 256;
__global__ __launch_bounds__(REDACT_BLOCK) void k_redact(const RulesDev R, const uint8_t* __restrict__ text,
                                                         const uint64_t* __restrict__ offs, uint32_t n_utt,
                                                         const pii_span* __restrict__ fd,
                                                         const uint32_t* __restrict__ n_find,
                                                         const uint64_t* __restrict__ out_offs,
                                                         const uint64_t* __restrict__ span_offs,
                                                         const uint32_t* __restrict__ err, uint8_t* __restrict__ out,
                                                         pii_span* __restrict__ spans,
                                                         unsigned long long* __restrict__ hist) {
    __shared__ uint32_t sh_hist[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) sh_hist[i] = 0;
    __syncthreads();
    const bool ok = *err == 0;
    const int lane = threadIdx.x & 63;
    const uint32_t u = blockIdx.x * (REDACT_BLOCK / 64) + (threadIdx.x >> 6);
    if (ok && u < n_utt) {
        const uint64_t base = offs[0];
        const uint64_t s_abs = offs[u], e_abs = offs[u + 1];
        const uint8_t* src = text + s_abs;
        const uint32_t nf = n_find[u];
        const pii_span* fdu = fd + (s_abs - base) / (uint64_t)R.min_len;
        uint8_t* dst = out + out_offs[u];
        pii_span* sp = spans + span_offs[u];
        uint32_t pos = 0;
        uint64_t o = 0;
        for (uint32_t f = 0; f < nf; ++f) {
            const pii_span F = fdu[f];
            for (uint32_t i = lane; i < F.start - pos; i += 64) dst[o + i] = src[pos + i];
            o += F.start - pos;
            const uint32_t t0 = R.tok_off[F.info_type], tl = R.tok_off[F.info_type + 1] - t0;
            for (uint32_t i = lane; i < tl; i += 64) dst[o + i] = R.tok_bytes[t0 + i];
            o += tl;
            pos = F.end;
            if (lane == 0) {
                sp[f] = F;
                if (F.info_type < 256) atomicAdd(&sh_hist[F.info_type], 1u);
            }
        }
        const uint32_t L = (uint32_t)(e_abs - s_abs);
        for (uint32_t i = lane; i < L - pos; i += 64) dst[o + i] = src[pos + i];
    }
    __syncthreads();
    if (ok) {
        for (int i = threadIdx.x; i < R.T && i < 256; i += blockDim.x)
            if (sh_hist[i]) atomicAdd(&hist[i], (unsigned long long)sh_hist[i]);
    }
}

__global__ void k_noop() {}

// ------------------------------------------------------------------------------- blob parsing
struct Section {
    std::string name;
    uint32_t dtype;
    const uint8_t* data;
    uint64_t bytes;
};

bool parse_blob(const uint8_t* p, size_t n, std::vector<Section>& out) {
    if (n < 12 || std::memcmp(p, "PIIRULE1", 8) != 0) return false;
    uint32_t cnt;
    std::memcpy(&cnt, p + 8, 4);
    size_t off = 12;
    for (uint32_t i = 0; i < cnt; ++i) {
        uint32_t ln;
        if (off + 4 > n) return false;
        std::memcpy(&ln, p + off, 4);
        off += 4;
        if (off + ln + 12 > n) return false;
        Section s;
        s.name.assign(reinterpret_cast<const char*>(p + off), ln);
        off += ln;
        std::memcpy(&s.dtype, p + off, 4);
        std::memcpy(&s.bytes, p + off + 4, 8);
        off += 12;
        if (off + s.bytes > n) return false;
        s.data = p + off;
        off += s.bytes;
        off += (8 - off % 8) % 8;
        out.push_back(s);
    }
    return true;
}

}  // namespace

// ================================================================================ engine object
struct pii_engine {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    RulesDev R{};
    void* d_rules = nullptr;
    std::vector<std::string> names;
    std::vector<int> kw_type;
    uint32_t n_slots = 0;
    int64_t ttl_us = 0;
    size_t scan_lds = 0;
    // persistent state (replaces Redis)
    int32_t* st_group = nullptr;
    int64_t* st_ts = nullptr;
    uint32_t* stamp = nullptr;
    uint32_t epoch = 0;
    unsigned long long* hist = nullptr;
    // scratch
    uint64_t cap_bytes = 0;
    uint32_t cap_utt = 0;
    Event* ev = nullptr;
    pii_span* fd = nullptr;
    uint32_t *n_ev = nullptr, *n_find = nullptr, *out_len = nullptr, *incl = nullptr, *agg_f = nullptr;
    uint32_t* first_utt = nullptr;
    int16_t *kw = nullptr, *ctx = nullptr;
    int32_t *agg_v = nullptr, *commit = nullptr;
    uint64_t *span_offs = nullptr, *bsum = nullptr, *out_offs_tmp = nullptr;
    uint32_t* d_err = nullptr;
    uint64_t* d_totals = nullptr;
    uint64_t* h_totals = nullptr;
    // host-API staging
    uint64_t cap_h_bytes = 0, cap_h_out = 0;
    uint32_t cap_h_utt = 0, cap_h_spans = 0;
    uint8_t *h_text = nullptr, *h_role = nullptr, *h_out = nullptr;
    uint64_t *h_offs = nullptr, *h_out_offs = nullptr;
    uint32_t* h_slot = nullptr;
    int64_t* h_ts = nullptr;
    pii_span* h_spans = nullptr;
    int16_t* h_ctx = nullptr;
    hipEvent_t tev[7] = {};
    float last_ms[6] = {};
};

#define HIPCHK(x)                                                                  \
    do {                                                                           \
        hipError_t _e = (x);                                                       \
        if (_e != hipSuccess) {                                                    \
            e->err = std::string(#x) + ": " + hipGetErrorString(_e);              \
            return PII_E_DEVICE;                                                   \
        }                                                                          \
    } while (0)

namespace {

template <class T>
int grow(pii_engine* e, T*& p, size_t count) {
    if (p) (void)hipFree(p);
    p = nullptr;
    if (count == 0) count = 1;
    if (hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)) != hipSuccess) {
        e->err = "device allocation failed";
        return PII_E_NOMEM;
    }
    return PII_OK;
}

int ensure_scratch(pii_engine* e, uint32_t n_utt, uint64_t bytes) {
    int rc = PII_OK;
    if (bytes > e->cap_bytes) {
        const uint64_t nb = std::max<uint64_t>(bytes + bytes / 8, 1 << 16);
        if ((rc = grow(e, e->ev, nb + 1))) return rc;
        if ((rc = grow(e, e->fd, nb / e->R.min_len + 2))) return rc;
        if ((rc = grow(e, e->first_utt, nb / BYTES_PER_LANE + 2))) return rc;
        e->cap_bytes = nb;
    }
    if (n_utt > e->cap_utt) {
        const uint32_t nu = std::max<uint32_t>(n_utt + n_utt / 8, 1024);
        if ((rc = grow(e, e->n_ev, nu))) return rc;
        if ((rc = grow(e, e->n_find, nu))) return rc;
        if ((rc = grow(e, e->out_len, nu))) return rc;
        if ((rc = grow(e, e->incl, nu))) return rc;
        if ((rc = grow(e, e->kw, nu))) return rc;
        if ((rc = grow(e, e->ctx, nu))) return rc;
        if ((rc = grow(e, e->commit, nu))) return rc;
        const uint32_t nblk = nu / CTX_BLOCK + 2;
        if ((rc = grow(e, e->agg_v, nblk))) return rc;
        if ((rc = grow(e, e->agg_f, nblk))) return rc;
        if ((rc = grow(e, e->span_offs, (size_t)nu + 1))) return rc;
        if ((rc = grow(e, e->out_offs_tmp, (size_t)nu + 1))) return rc;
        if ((rc = grow(e, e->bsum, (size_t)nu / SCAN_TILE + 2))) return rc;
        e->cap_utt = nu;
    }
    return rc;
}

int exclusive_scan(pii_engine* e, const uint32_t* in, uint32_t n, uint64_t* out, hipStream_t st) {
    const uint32_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 0) {
        HIPCHK(hipMemsetAsync(out, 0, sizeof(uint64_t), st));
        return PII_OK;
    }
    k_scan_reduce<<<nb, 256, 0, st>>>(in, n, e->bsum);
    k_scan_blocks<<<1, 256, 0, st>>>(e->bsum, nb);
    k_scan_apply<<<nb, 256, 0, st>>>(in, n, e->bsum, out);
    HIPCHK(hipGetLastError());
    return PII_OK;
}

int run_pipeline(pii_engine* e, const uint8_t* text, const uint64_t* offs, uint32_t n_utt, uint64_t total_bytes,
                 const uint32_t* slot, const uint8_t* role, const int64_t* ts, uint8_t* out, uint64_t out_cap,
                 uint64_t* out_offs, pii_span* spans, uint32_t span_cap, int16_t* ctx_info, hipStream_t st) {
    int rc = ensure_scratch(e, n_utt, total_bytes);
    if (rc) return rc;
    const RulesDev& R = e->R;
    e->epoch += 1;
    HIPCHK(hipMemsetAsync(e->d_err, 0, sizeof(uint32_t), st));
    HIPCHK(hipEventRecord(e->tev[0], st));
    const uint32_t n_chunks = (uint32_t)((total_bytes + BYTES_PER_LANE - 1) / BYTES_PER_LANE);
    if (n_utt > 0) {
        k_chunk_index<<<(n_utt + 1 + 255) / 256, 256, 0, st>>>(offs, n_utt, n_chunks, e->first_utt);
        if (n_chunks > 0)
            k_scan<<<(n_chunks + SCAN_BLOCK - 1) / SCAN_BLOCK, SCAN_BLOCK, e->scan_lds, st>>>(
                R, text, offs, n_utt, role, e->first_utt, n_chunks, e->ev, e->n_ev, e->kw);
        else
            HIPCHK(hipMemsetAsync(e->n_ev, 0, n_utt * sizeof(uint32_t), st));
        if (n_chunks == 0) {
            // all rows empty: no scan ran, so fill keyword results directly
            std::vector<int16_t> none(n_utt, -1);
            HIPCHK(hipMemcpyAsync(e->kw, none.data(), n_utt * sizeof(int16_t), hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(e->tev[1], st));
    const uint32_t nblk = (n_utt + CTX_BLOCK - 1) / CTX_BLOCK;
    if (n_utt > 0) {
        k_ctx_scan<<<nblk, CTX_BLOCK, 0, st>>>(slot, role, e->kw, n_utt, e->n_slots, e->incl, e->agg_v, e->agg_f,
                                               e->stamp, e->epoch, e->d_err);
        k_ctx_apply<<<(n_utt + 255) / 256, 256, 0, st>>>(slot, role, e->kw, ts, n_utt, e->n_slots, e->ttl_us,
                                                         e->incl, e->agg_v, e->agg_f, e->st_group, e->st_ts,
                                                         ctx_info ? ctx_info : e->ctx, e->commit);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(e->tev[2], st));
    if (n_utt > 0) {
        k_resolve<<<(n_utt + 255) / 256, 256, 0, st>>>(R, text, offs, n_utt, role, ctx_info ? ctx_info : e->ctx,
                                                      e->ev, e->n_ev, e->fd, e->n_find, e->out_len);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(e->tev[3], st));
    if ((rc = exclusive_scan(e, e->out_len, n_utt, out_offs, st))) return rc;
    if ((rc = exclusive_scan(e, e->n_find, n_utt, e->span_offs, st))) return rc;
    k_finalize<<<1, 1, 0, st>>>(out_offs, e->span_offs, n_utt, out_cap, span_cap, e->d_err, e->d_totals);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(e->tev[4], st));
    if (n_utt > 0) {
        k_redact<<<(n_utt + REDACT_BLOCK / 64 - 1) / (REDACT_BLOCK / 64), REDACT_BLOCK, 0, st>>>(
            R, text, offs, n_utt, e->fd, e->n_find, out_offs, e->span_offs, e->d_err, out, spans, e->hist);
        k_ctx_commit<<<(n_utt + 255) / 256, 256, 0, st>>>(slot, e->kw, ts, n_utt, e->n_slots, e->commit, e->d_err,
                                                          e->st_group, e->st_ts);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(e->tev[5], st));
    HIPCHK(hipMemcpyAsync(e->h_totals, e->d_totals, 3 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(e->tev[6], st));
    return PII_OK;
}

}  // namespace

extern "C" {

const char* pii_last_error(pii_engine* e) { return e ? e->err.c_str() : "null engine"; }

int pii_engine_create(const void* blob, size_t n, int device, uint32_t n_conv_slots, int64_t ttl_us,
                      pii_engine** out) {
    if (!blob || !out) return PII_E_ARG;
    *out = nullptr;
    std::vector<Section> secs;
    if (!parse_blob(static_cast<const uint8_t*>(blob), n, secs)) return PII_E_RULES;
    auto find = [&](const char* nm) -> const Section* {
        for (auto& s : secs)
            if (s.name == nm) return &s;
        return nullptr;
    };
    static const char* req[] = {"meta", "scan.cmap2", "scan.d.trans", "scan.d.accid", "scan.d.acc_off",
                                "scan.d.acc_ids", "scan.k.trans", "scan.k.accid", "scan.k.acc_off", "scan.k.acc_ids",
                                "det.type", "det.validator", "det.lik", "det.exidx", "det.first_desc", "hot.rule",
                                "hot.dfa_desc", "pool.trans", "pool.flags", "pool.cmap", "var.enabled",
                                "var.minlik", "var.rule_off", "var.rule_ids", "var.excl_off", "var.excl_ids",
                                "kw.type", "kw.always", "types.names"};
    for (auto r : req)
        if (!find(r)) return PII_E_RULES;
    const int64_t* meta = reinterpret_cast<const int64_t*>(find("meta")->data);
    pii_engine* e = new pii_engine();
    e->device = device;
    e->n_slots = n_conv_slots;
    e->ttl_us = ttl_us;
    RulesDev& R = e->R;
    R.P = (int)meta[0];
    R.G = (int)meta[1];
    R.T = (int)meta[2];
    R.V = (int)meta[3];
    R.SD = (int)meta[4];
    R.CD = (int)meta[5];
    R.d_start = (int)meta[6];
    R.SK = (int)meta[7];
    R.CK = (int)meta[8];
    R.k_start = (int)meta[9];
    R.n_hot = (int)meta[10];
    R.min_len = (int)std::max<int64_t>(1, meta[11]);
    auto fail = [&](const char* why) {
        e->err = why;
        pii_engine_destroy(e);
        return PII_E_RULES;
    };
    if (R.P > P_MAX) return fail("more detector patterns than P_MAX");
    if ((int64_t)R.SD * R.CD >= 32768 || (int64_t)R.SK * R.CK >= 32768) return fail("SCAN tables exceed 15-bit rows");
    if (R.T > 65535) return fail("too many types");
    // names + tokens
    {
        const Section* s = find("types.names");
        const char* p = reinterpret_cast<const char*>(s->data);
        size_t i = 0;
        while (i < s->bytes) {
            size_t l = strnlen(p + i, s->bytes - i);
            e->names.emplace_back(p + i, l);
            i += l + 1;
        }
        if ((int)e->names.size() != R.T) return fail("type table mismatch");
    }
    {
        const Section* s = find("kw.type");
        const uint16_t* k = reinterpret_cast<const uint16_t*>(s->data);
        for (int g = 0; g < R.G; ++g) e->kw_type.push_back(k[g]);
    }
    // host-side derived tables
    std::vector<uint16_t> td(R.SD * R.CD), tk(R.SK * R.CK);
    {
        const uint16_t* s = reinterpret_cast<const uint16_t*>(find("scan.d.trans")->data);
        for (int i = 0; i < R.SD * R.CD; ++i) td[i] = (uint16_t)(((s[i] & 0x7fff) * R.CD) | (s[i] & 0x8000));
        const uint16_t* k = reinterpret_cast<const uint16_t*>(find("scan.k.trans")->data);
        for (int i = 0; i < R.SK * R.CK; ++i) tk[i] = (uint16_t)(((k[i] & 0x7fff) * R.CK) | (k[i] & 0x8000));
    }
    std::vector<uint16_t> k_acc_min;
    {
        const Section* so = find("scan.k.acc_off");
        const uint32_t* off = reinterpret_cast<const uint32_t*>(so->data);
        const uint16_t* ids = reinterpret_cast<const uint16_t*>(find("scan.k.acc_ids")->data);
        const size_t nsets = so->bytes / 4 - 1;
        for (size_t a = 0; a < nsets; ++a) {
            int m = KW_NONE;
            for (uint32_t i = off[a]; i < off[a + 1]; ++i) m = std::min<int>(m, ids[i]);
            k_acc_min.push_back((uint16_t)m);
        }
    }
    R.kw_always_min = KW_NONE;
    {
        const uint8_t* al = find("kw.always")->data;
        for (int g = 0; g < R.G; ++g)
            if (al[g]) {
                R.kw_always_min = g;
                break;
            }
    }
    {
        const uint8_t* ex = find("det.exidx")->data;
        int ne = 0;
        for (int p = 0; p < R.P; ++p)
            if (ex[p] != 0xff) ne = std::max(ne, ex[p] + 1);
        if (ne > NE_MAX) return fail("too many excluder patterns");
        R.NE = ne;
    }
    std::vector<uint32_t> tok_off(R.T + 1, 0);
    std::string tok;
    for (int t = 0; t < R.T; ++t) {
        tok += "[" + e->names[t] + "]";
        tok_off[t + 1] = (uint32_t)tok.size();
    }
    // one device buffer holding every table, 256-byte aligned sections
    struct Put {
        const void* src;
        size_t bytes;
        size_t off;
    };
    std::vector<Put> puts;
    size_t total = 0;
    auto add = [&](const void* src, size_t bytes) {
        total = (total + 255) & ~(size_t)255;
        puts.push_back({src, bytes, total});
        total += bytes + 16;
        return puts.size() - 1;
    };
    auto addsec = [&](const char* nm) { return add(find(nm)->data, find(nm)->bytes); };
    size_t i_cmap = addsec("scan.cmap2"), i_td = add(td.data(), td.size() * 2), i_tk = add(tk.data(), tk.size() * 2);
    size_t i_dacc = addsec("scan.d.accid"), i_doff = addsec("scan.d.acc_off"), i_dids = addsec("scan.d.acc_ids");
    size_t i_kacc = addsec("scan.k.accid"), i_kmin = add(k_acc_min.data(), k_acc_min.size() * 2);
    size_t i_dt = addsec("det.type"), i_dv = addsec("det.validator"), i_dl = addsec("det.lik"),
           i_dx = addsec("det.exidx"), i_fd = addsec("det.first_desc"), i_hr = addsec("hot.rule"),
           i_hd = addsec("hot.dfa_desc"), i_pt = addsec("pool.trans"), i_pf = addsec("pool.flags"),
           i_pc = addsec("pool.cmap"), i_ve = addsec("var.enabled"), i_vm = addsec("var.minlik"),
           i_ro = addsec("var.rule_off"), i_ri = addsec("var.rule_ids"), i_eo = addsec("var.excl_off"),
           i_ei = addsec("var.excl_ids"), i_to = add(tok_off.data(), tok_off.size() * 4),
           i_tb = add(tok.data(), tok.size());
    if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice failed");
    if (hipMalloc(&e->d_rules, total) != hipSuccess) return fail("hipMalloc rules failed");
    std::vector<uint8_t> host(total, 0);
    for (auto& p : puts) std::memcpy(host.data() + p.off, p.src, p.bytes);
    if (hipMemcpy(e->d_rules, host.data(), total, hipMemcpyHostToDevice) != hipSuccess) return fail("upload failed");
    uint8_t* b = static_cast<uint8_t*>(e->d_rules);
    auto at = [&](size_t i) { return b + puts[i].off; };
    R.cmap2 = (const uint16_t*)at(i_cmap);
    R.td = (const uint16_t*)at(i_td);
    R.tk = (const uint16_t*)at(i_tk);
    R.d_accid = (const uint16_t*)at(i_dacc);
    R.d_acc_off = (const uint32_t*)at(i_doff);
    R.d_acc_ids = (const uint16_t*)at(i_dids);
    R.k_accid = (const uint16_t*)at(i_kacc);
    R.k_acc_min = (const uint16_t*)at(i_kmin);
    R.det_type = (const uint16_t*)at(i_dt);
    R.det_val = (const uint8_t*)at(i_dv);
    R.det_lik = (const uint8_t*)at(i_dl);
    R.det_exidx = (const uint8_t*)at(i_dx);
    R.first_desc = (const int32_t*)at(i_fd);
    R.hot_rule = (const int32_t*)at(i_hr);
    R.hot_desc = (const int32_t*)at(i_hd);
    R.pool.trans = (const uint16_t*)at(i_pt);
    R.pool.flags = (const uint8_t*)at(i_pf);
    R.pool.cmap = (const uint8_t*)at(i_pc);
    R.var_enabled = (const uint8_t*)at(i_ve);
    R.var_minlik = (const uint8_t*)at(i_vm);
    R.rule_off = (const uint32_t*)at(i_ro);
    R.rule_ids = (const uint16_t*)at(i_ri);
    R.excl_off = (const uint32_t*)at(i_eo);
    R.excl_ids = (const uint16_t*)at(i_ei);
    R.tok_off = (const uint32_t*)at(i_to);
    R.tok_bytes = (const uint8_t*)at(i_tb);
    e->scan_lds = 512 + (size_t)((R.SD * R.CD + 1) / 2) * 4 + (size_t)((R.SK * R.CK + 1) / 2) * 4;
    if (e->scan_lds > 160 * 1024) return fail("SCAN tables do not fit in LDS");
    if (e->scan_lds > 64 * 1024 &&
        hipFuncSetAttribute((const void*)k_scan, hipFuncAttributeMaxDynamicSharedMemorySize, (int)e->scan_lds) != hipSuccess)
        return fail("cannot raise LDS limit");
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return fail("stream");
    e->own_stream = true;
    for (auto& t : e->tev)
        if (hipEventCreate(&t) != hipSuccess) return fail("event");
    const size_t ns = std::max<uint32_t>(1, n_conv_slots);
    if (hipMalloc(&e->st_group, ns * 4) != hipSuccess || hipMalloc(&e->st_ts, ns * 8) != hipSuccess ||
        hipMalloc(&e->stamp, ns * 4) != hipSuccess || hipMalloc(&e->hist, 256 * 8) != hipSuccess ||
        hipMalloc(&e->d_err, 16) != hipSuccess || hipMalloc(&e->d_totals, 64) != hipSuccess)
        return fail("state allocation failed");
    if (hipHostMalloc(&e->h_totals, 64) != hipSuccess) return fail("pinned allocation failed");
    std::vector<int32_t> g(ns, -1);
    if (hipMemcpy(e->st_group, g.data(), ns * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(e->st_ts, 0, ns * 8) != hipSuccess || hipMemset(e->stamp, 0, ns * 4) != hipSuccess ||
        hipMemset(e->hist, 0, 256 * 8) != hipSuccess)
        return fail("state init failed");
    k_noop<<<1, 64, 0, e->stream>>>();
    if (hipStreamSynchronize(e->stream) != hipSuccess) return fail("device not usable");
    *out = e;
    return PII_OK;
}

int pii_engine_destroy(pii_engine* e) {
    if (!e) return PII_E_ARG;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    void* ptrs[] = {e->d_rules, e->st_group, e->st_ts, e->stamp, e->hist, e->ev, e->fd, e->n_ev, e->n_find,
                    e->out_len, e->incl, e->agg_f, e->first_utt, e->kw, e->ctx, e->agg_v, e->commit,
                    e->span_offs, e->bsum, e->out_offs_tmp, e->d_err, e->d_totals, e->h_text, e->h_role,
                    e->h_out, e->h_offs, e->h_out_offs, e->h_slot, e->h_ts, e->h_spans, e->h_ctx};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (e->h_totals) (void)hipHostFree(e->h_totals);
    for (auto& t : e->tev)
        if (t) (void)hipEventDestroy(t);
    if (e->stream && e->own_stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return PII_OK;
}

int pii_engine_info(pii_engine* e, pii_info* out) {
    if (!e || !out) return PII_E_ARG;
    out->n_types = (uint32_t)e->R.T;
    out->n_patterns = (uint32_t)e->R.P;
    out->n_context_groups = (uint32_t)e->R.G;
    out->n_conv_slots = e->n_slots;
    out->scan_states_d = (uint32_t)e->R.SD;
    out->scan_states_k = (uint32_t)e->R.SK;
    out->scan_lds_bytes = (uint32_t)e->scan_lds;
    out->reserved = 0;
    return PII_OK;
}

int pii_type_name(pii_engine* e, uint32_t t, char* buf, size_t cap) {
    if (!e || t >= e->names.size()) return PII_E_ARG;
    const std::string& s = e->names[t];
    if (buf && cap) {
        const size_t n = std::min(cap - 1, s.size());
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int)s.size();
}

int pii_context_group_type(pii_engine* e, uint32_t g) {
    if (!e || g >= e->kw_type.size()) return PII_E_ARG;
    return e->kw_type[g];
}

int pii_scan_redact_device(pii_engine* e, const uint8_t* d_bytes, const uint64_t* d_offsets, uint32_t n_utt,
                           const uint32_t* d_slot, const uint8_t* d_role, const int64_t* d_ts, uint8_t* d_out,
                           uint64_t out_cap, uint64_t* d_out_offsets, pii_span* d_spans, uint32_t span_cap,
                           int16_t* d_ctx_info, void* stream) {
    if (!e || !d_offsets || !d_slot || !d_role || !d_out_offsets) return PII_E_ARG;
    if (n_utt > 0 && (!d_bytes || !d_out || !d_spans)) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : e->stream;
    uint64_t tb[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(tb, d_offsets, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(tb + 1, d_offsets + n_utt, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    if (tb[1] < tb[0]) return PII_E_ARG;
    return run_pipeline(e, d_bytes, d_offsets, n_utt, tb[1] - tb[0], d_slot, d_role, d_ts, d_out, out_cap,
                        d_out_offsets, d_spans, span_cap, d_ctx_info, st);
}

int pii_sync(pii_engine* e, uint64_t totals[3]) {
    if (!e) return PII_E_ARG;
    HIPCHK(hipEventSynchronize(e->tev[6]));
    const char* names[] = {"scan", "context", "resolve", "offsets", "redact"};
    (void)names;
    float tot = 0;
    for (int i = 0; i < 5; ++i) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e->tev[i], e->tev[i + 1]));
        e->last_ms[i] = ms;
        tot += ms;
    }
    e->last_ms[5] = tot;
    if (totals) {
        totals[0] = e->h_totals[0];
        totals[1] = e->h_totals[1];
        totals[2] = e->h_totals[2];
    }
    const uint64_t f = e->h_totals[2];
    if (f & ERR_SLOT) return PII_E_ARG;
    if (f & ERR_ORDER) return PII_E_ORDER;
    if (f & ERR_CAPACITY) return PII_E_CAPACITY;
    return PII_OK;
}

int pii_last_timings(pii_engine* e, float ms[6]) {
    if (!e || !ms) return PII_E_ARG;
    std::memcpy(ms, e->last_ms, sizeof(e->last_ms));
    return PII_OK;
}

int pii_scan_redact(pii_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint32_t n_utt,
                    const uint32_t* conv_slot, const uint8_t* role, const int64_t* ts_us, uint8_t* out_bytes,
                    uint64_t out_cap, uint64_t* out_offsets, pii_span* spans, uint32_t span_cap, uint32_t* n_spans,
                    int16_t* ctx_info) {
    if (!e || !offsets || !out_offsets || (n_utt && (!conv_slot || !role))) return PII_E_ARG;
    for (uint32_t i = 0; i < n_utt; ++i)
        if (offsets[i + 1] < offsets[i]) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    const uint64_t base = offsets[0], total = offsets[n_utt] - base;
    int rc;
    if (total + 16 > e->cap_h_bytes) {
        const uint64_t nb = total + total / 8 + 64;
        if ((rc = grow(e, e->h_text, nb))) return rc;
        e->cap_h_bytes = nb;
    }
    if (n_utt + 1 > e->cap_h_utt) {
        const uint32_t nu = n_utt + n_utt / 8 + 64;
        if ((rc = grow(e, e->h_offs, nu + 1)) || (rc = grow(e, e->h_out_offs, nu + 1)) ||
            (rc = grow(e, e->h_slot, nu)) || (rc = grow(e, e->h_role, nu)) || (rc = grow(e, e->h_ts, nu)) ||
            (rc = grow(e, e->h_ctx, nu)))
            return rc;
        e->cap_h_utt = nu;
    }
    if (out_cap + 16 > e->cap_h_out) {
        const uint64_t nb = out_cap + 64;
        if ((rc = grow(e, e->h_out, nb))) return rc;
        e->cap_h_out = nb;
    }
    if (span_cap + 1 > e->cap_h_spans) {
        const uint32_t ns = span_cap + 64;
        if ((rc = grow(e, e->h_spans, ns))) return rc;
        e->cap_h_spans = ns;
    }
    hipStream_t st = e->stream;
    std::vector<uint64_t> rel(n_utt + 1);
    for (uint32_t i = 0; i <= n_utt; ++i) rel[i] = offsets[i] - base;
    if (total) HIPCHK(hipMemcpyAsync(e->h_text, bytes + base, total, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(e->h_offs, rel.data(), (n_utt + 1) * 8, hipMemcpyHostToDevice, st));
    if (n_utt) {
        HIPCHK(hipMemcpyAsync(e->h_slot, conv_slot, n_utt * 4, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(e->h_role, role, n_utt, hipMemcpyHostToDevice, st));
        if (ts_us) HIPCHK(hipMemcpyAsync(e->h_ts, ts_us, n_utt * 8, hipMemcpyHostToDevice, st));
    }
    rc = run_pipeline(e, e->h_text, e->h_offs, n_utt, total, e->h_slot, e->h_role, ts_us ? e->h_ts : nullptr,
                      e->h_out, out_cap, e->h_out_offs, e->h_spans, span_cap, e->h_ctx, st);
    if (rc) return rc;
    uint64_t tot[3];
    rc = pii_sync(e, tot);
    if (rc == PII_E_CAPACITY) {
        HIPCHK(hipMemcpy(out_offsets, e->h_out_offs, (n_utt + 1) * 8, hipMemcpyDeviceToHost));
        if (n_spans) *n_spans = (uint32_t)tot[1];
        return rc;
    }
    if (rc) return rc;
    HIPCHK(hipMemcpy(out_offsets, e->h_out_offs, (n_utt + 1) * 8, hipMemcpyDeviceToHost));
    if (tot[0]) HIPCHK(hipMemcpy(out_bytes, e->h_out, tot[0], hipMemcpyDeviceToHost));
    if (tot[1]) HIPCHK(hipMemcpy(spans, e->h_spans, tot[1] * sizeof(pii_span), hipMemcpyDeviceToHost));
    if (n_spans) *n_spans = (uint32_t)tot[1];
    if (ctx_info && n_utt) HIPCHK(hipMemcpy(ctx_info, e->h_ctx, n_utt * 2, hipMemcpyDeviceToHost));
    return PII_OK;
}

int pii_context_get(pii_engine* e, uint32_t slot, int32_t* group, int64_t* ts_us) {
    if (!e || slot >= e->n_slots) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    int32_t g;
    int64_t t;
    HIPCHK(hipMemcpy(&g, e->st_group + slot, 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&t, e->st_ts + slot, 8, hipMemcpyDeviceToHost));
    if (group) *group = g;
    if (ts_us) *ts_us = t;
    return PII_OK;
}

int pii_context_set(pii_engine* e, uint32_t slot, int32_t group, int64_t ts_us) {
    if (!e || slot >= e->n_slots || group < -1 || group >= e->R.G) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    HIPCHK(hipMemcpy(e->st_group + slot, &group, 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(e->st_ts + slot, &ts_us, 8, hipMemcpyHostToDevice));
    return PII_OK;
}

int pii_histogram(pii_engine* e, uint64_t* counts, uint32_t n) {
    if (!e || !counts) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipStreamSynchronize(e->stream));
    std::vector<unsigned long long> h(256);
    HIPCHK(hipMemcpy(h.data(), e->hist, 256 * 8, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) counts[i] = i < 256 ? h[i] : 0;
    return PII_OK;
}

int pii_histogram_reset(pii_engine* e) {
    if (!e) return PII_E_ARG;
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemsetAsync(e->hist, 0, 256 * 8, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return PII_OK;
}

}  // extern "C"

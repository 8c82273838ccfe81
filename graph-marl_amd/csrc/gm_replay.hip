// gm_replay.hip — replay-memory sampling stream of the reference on the device.
//
// The reference samples its replay with np.random.default_rng(seed).choice(n, size,
// replace=True) (src/replaybuffer.py:101-130), i.e. numpy's Generator (numpy >= 1.17, the
// algorithm unchanged since; pinned against the numpy of this image by tests/test_replay_rng.py):
//   * seeding: SeedSequence(seed).generate_state(4, uint64) -> PCG64 seed (hi, lo) and
//     increment (hi, lo); pcg_setseq_128_srandom_r (state 0, inc = 2 seq + 1, step, += seed, step);
//   * PCG64 (XSL-RR 128/64): state = state * M + inc, out = rotr64(hi ^ lo, state >> 122);
//     32-bit draws use both halves of an output, low half first, the high half buffered in the
//     generator (has_uint32 / uinteger carry over between calls);
//   * choice(n, k) = integers(0, n, k, int64): for n - 1 < 2^32 - 1, Lemire's bounded draw per
//     element: m = u32 * n, reject while (m mod 2^32) < (2^32 - n) mod n, value = m >> 32.
// Device form: one workgroup of 1024 threads walks the output in chunks of 1024 draws. Thread t
// computes the t-th 32-bit draw of the chunk directly by jumping the LCG ahead (O(log t) 128-bit
// multiply-adds), so a chunk costs one jump per thread instead of a 1024-long dependent chain.
// Rejections (probability (2^32 mod n) / 2^32 per draw, < 3e-5 for replay sizes) are resolved
// exactly: the chunk keeps the draws before the first rejecting one, thread 0 finishes that
// element sequentially (redraws as numpy does), and the next chunk starts after it. The
// generator state lives in device memory and is advanced in place (no host round trip).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "../../include/graph_marl_amd.h"

int gm_fail(int code, const std::string& msg);

namespace {

typedef unsigned __int128 u128;

constexpr uint64_t PCG_MULT_HI = 2549297995355413924ULL, PCG_MULT_LO = 4865540595714422341ULL;

__host__ __device__ inline u128 mk(uint64_t hi, uint64_t lo) { return ((u128)hi << 64) | lo; }

__host__ __device__ inline uint64_t xsl_rr(u128 s) {
    const uint64_t x = (uint64_t)(s >> 64) ^ (uint64_t)s;
    const unsigned r = (unsigned)(s >> 122);
    return (x >> r) | (x << ((64u - r) & 63u));
}

// state after k LCG steps (pcg_advance_lcg_128)
__device__ inline u128 advance(u128 s, u128 inc, uint64_t k) {
    u128 cur_mult = mk(PCG_MULT_HI, PCG_MULT_LO), cur_plus = inc, acc_mult = 1, acc_plus = 0;
    while (k) {
        if (k & 1) {
            acc_mult *= cur_mult;
            acc_plus = acc_plus * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        k >>= 1;
    }
    return acc_mult * s + acc_plus;
}

struct Pos {  // position in the 32-bit draw stream
    u128 s;   // state after the last 64-bit output taken
    unsigned has, u;
};

// the d-th (0-based) 32-bit draw from position p
__device__ inline unsigned draw_at(const Pos& p, u128 inc, uint64_t d) {
    if (p.has) {
        if (d == 0) return p.u;
        d -= 1;
    }
    const uint64_t x = xsl_rr(advance(p.s, inc, d / 2 + 1));
    return (d & 1) ? (unsigned)(x >> 32) : (unsigned)x;
}

// position after d draws
__device__ inline Pos skip(Pos p, u128 inc, uint64_t d) {
    if (d == 0) return p;
    if (p.has) {
        p.has = 0;
        d -= 1;
        if (d == 0) return p;
    }
    p.s = advance(p.s, inc, (d + 1) / 2);
    p.u = (unsigned)(xsl_rr(p.s) >> 32);  // numpy keeps the last output's high half, consumed or not
    p.has = d & 1;
    return p;
}

__device__ inline unsigned next32(Pos& p, u128 inc) {
    if (p.has) {
        p.has = 0;
        return p.u;
    }
    p.s = p.s * mk(PCG_MULT_HI, PCG_MULT_LO) + inc;
    const uint64_t x = xsl_rr(p.s);
    p.has = 1;
    p.u = (unsigned)(x >> 32);
    return (unsigned)x;
}

constexpr int CH = 1024;

__global__ __launch_bounds__(CH) void k_pcg64_choice(gm_pcg64* __restrict__ g, uint32_t n, unsigned threshold,
                                                    long long count, long long* __restrict__ out) {
    __shared__ Pos pos;
    __shared__ int first_bad;
    __shared__ long long done;
    const int t = threadIdx.x;
    const u128 inc = mk(g->inc_hi, g->inc_lo);
    if (t == 0) {
        pos.s = mk(g->state_hi, g->state_lo);
        pos.has = g->has_uint32;
        pos.u = g->uinteger;
        done = 0;
    }
    __syncthreads();
    while (true) {
        const long long base = done;
        if (base >= count) break;
        const int len = (int)min((long long)CH, count - base);
        if (t == 0) first_bad = CH;
        __syncthreads();
        unsigned long long m = 0;
        if (t < len) {
            m = (unsigned long long)draw_at(pos, inc, (uint64_t)t) * n;
            if ((unsigned)m < threshold) atomicMin(&first_bad, t);  // LDS atomic
        }
        __syncthreads();
        const int v = min(first_bad, len);  // draws accepted without a redraw
        if (t < v) out[base + t] = (long long)(m >> 32);
        __syncthreads();
        if (t == 0) {
            Pos p = skip(pos, inc, (uint64_t)v);
            long long nd = base + v;
            if (v < len) {  // element v: numpy's rejection loop, sequentially
                unsigned long long mm;
                do {
                    mm = (unsigned long long)next32(p, inc) * n;
                } while ((unsigned)mm < threshold);
                out[nd] = (long long)(mm >> 32);
                nd += 1;
            }
            pos = p;
            done = nd;
        }
        __syncthreads();
    }
    if (t == 0) {
        g->state_hi = (uint64_t)(pos.s >> 64);
        g->state_lo = (uint64_t)pos.s;
        g->has_uint32 = pos.has;
        g->uinteger = pos.u;
    }
}

// ---- SeedSequence (numpy/random/bit_generator.pyx), host side ----
constexpr uint32_t INIT_A = 0x43b0d7e5u, MULT_A = 0x931e8875u, INIT_B = 0x8b51f9ddu, MULT_B = 0x58f38dedu;
constexpr uint32_t MIX_L = 0xca01f9ddu, MIX_R = 0x4973f715u;

uint32_t hashmix(uint32_t v, uint32_t& hc) {
    v ^= hc;
    hc *= MULT_A;
    v *= hc;
    v ^= v >> 16;
    return v;
}

uint32_t mix(uint32_t x, uint32_t y) {
    uint32_t r = MIX_L * x - MIX_R * y;
    r ^= r >> 16;
    return r;
}

}  // namespace

extern "C" int gm_pcg64_seed(uint64_t seed, gm_pcg64* out) {
    if (!out) return gm_fail(GM_ERR_INVALID_ARG, "gm_pcg64_seed: null output");
    // entropy: the seed as little-endian 32-bit words (at least one)
    uint32_t ent[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const int ne = (seed >> 32) ? 2 : 1;
    uint32_t pool[4];
    uint32_t hc = INIT_A;
    for (int i = 0; i < 4; i++) pool[i] = hashmix(i < ne ? ent[i] : 0u, hc);
    for (int s = 0; s < 4; s++)
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = mix(pool[d], hashmix(pool[s], hc));
    uint32_t w[8];
    uint32_t hb = INIT_B;
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= MULT_B;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    uint64_t v64[4];
    for (int i = 0; i < 4; i++) v64[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
    const u128 s0 = mk(v64[0], v64[1]), seq = mk(v64[2], v64[3]);
    const u128 M = mk(PCG_MULT_HI, PCG_MULT_LO);
    const u128 inc = (seq << 1) | 1;
    u128 st = 0;
    st = st * M + inc;
    st += s0;
    st = st * M + inc;
    out->state_hi = (uint64_t)(st >> 64);
    out->state_lo = (uint64_t)st;
    out->inc_hi = (uint64_t)(inc >> 64);
    out->inc_lo = (uint64_t)inc;
    out->has_uint32 = 0;
    out->uinteger = 0;
    return GM_OK;
}

extern "C" int gm_pcg64_choice(gm_pcg64* state, int64_t n, int64_t count, int64_t* out, void* stream) {
    if (!state || (count > 0 && !out) || count < 0 || n < 1)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_pcg64_choice: bad arguments (n >= 1, count >= 0)");
    if (n > 0xFFFFFFFFLL)
        return gm_fail(GM_ERR_UNSUPPORTED, "gm_pcg64_choice: n > 2^32 - 1 (numpy's 64-bit Lemire path)");
    if (count == 0) return GM_OK;
    if (n == 1) {  // rng == 0: no draw, every value 0
        if (hipMemsetAsync(out, 0, (size_t)count * 8, (hipStream_t)stream) != hipSuccess)
            return gm_fail(GM_ERR_HIP, "gm_pcg64_choice: memset failed");
        return GM_OK;
    }
    const uint32_t nn = (uint32_t)n;
    const unsigned threshold = (unsigned)((0x100000000ULL - nn) % nn);
    hipLaunchKernelGGL(k_pcg64_choice, dim3(1), dim3(CH), 0, (hipStream_t)stream, state, nn, threshold,
                       (long long)count, reinterpret_cast<long long*>(out));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_pcg64_choice launch: ") + hipGetErrorString(e));
    return GM_OK;
}

// ---- sampled-field gather (replaybuffer.get_sequences): dst row i = the (slot[i], env[i % n_env_idx])
// record of a ring field, `bytes` (a multiple of 16) per record. The records of a sampled batch are
// scattered KB-sized blocks; the flattened float4 index space is split into 1024-float4 chunks per
// workgroup with U loads in flight per thread (torch's advanced indexing reads them at ~1.9 TB/s).
constexpr int GU = 4;
__global__ __launch_bounds__(256) void k_gather_records(const char* __restrict__ src, long long ld_slot,
                                                        long long ld_env, const long long* __restrict__ slot,
                                                        const long long* __restrict__ env, int n_env_idx,
                                                        unsigned total, unsigned q, float4* __restrict__ dst) {
    const unsigned base = blockIdx.x * (256u * GU) + threadIdx.x;
    float4 v[GU];
#pragma unroll
    for (int u = 0; u < GU; u++) {
        const unsigned e = base + u * 256u;
        if (e < total) {
            const unsigned r = e / q, c = e - r * q;
            const long long off = slot[r] * ld_slot + env[r % (unsigned)n_env_idx] * ld_env;
            v[u] = *reinterpret_cast<const float4*>(src + off + 16ll * c);
        }
    }
#pragma unroll
    for (int u = 0; u < GU; u++) {
        const unsigned e = base + u * 256u;
        if (e < total) dst[e] = v[u];
    }
}

extern "C" int gm_gather_records(const void* src, int64_t ld_slot, int64_t ld_env, const int64_t* slot,
                                 const int64_t* env, int32_t n_env_idx, int64_t n, int64_t bytes, void* dst,
                                 void* stream) {
    if (!src || !slot || !env || !dst || n < 0 || n_env_idx <= 0 || bytes <= 0 || (bytes & 15) || (ld_slot & 15) ||
        (ld_env & 15) || (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_gather_records: bad arguments (16-byte records, strides, bases)");
    const long long q = bytes / 16;
    if (n == 0) return GM_OK;
    if (n * q >= (1ll << 31) - 256ll * GU)
        return gm_fail(GM_ERR_UNSUPPORTED, "gm_gather_records: more than 2^31 float4 per call");
    const unsigned total = (unsigned)(n * q);
    const unsigned blocks = (total + 256u * GU - 1) / (256u * GU);
    hipLaunchKernelGGL(k_gather_records, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const char*>(src), (long long)ld_slot, (long long)ld_env,
                       reinterpret_cast<const long long*>(slot), reinterpret_cast<const long long*>(env), n_env_idx,
                       total, (unsigned)q, static_cast<float4*>(dst));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("gm_gather_records launch: ") + hipGetErrorString(e));
    return GM_OK;
}

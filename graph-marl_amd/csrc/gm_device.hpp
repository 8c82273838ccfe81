// gm_device.hpp — wave-level helpers and the numpy-legacy MT19937 stream on gfx950.
//
// Every env kernel runs ONE 64-lane wavefront per environment (blockDim = 64).
// "Uniform" code paths are executed by all lanes in lockstep with identical
// values (the compiler keeps them in SGPRs), so sequential reference semantics
// (packet-id order, RNG draw order) need no lane-0 special-casing or broadcasts.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gm {

constexpr int WAVE = 64;
constexpr int MT_N = 624;
constexpr int MT_M = 397;
constexpr int MAX_NODES = 128;  // node-indexed work runs in lanes v = l, l + 64
constexpr int MAX_AGENTS = 64;
constexpr int MAX_KNBR = 8;     // neighbour slots of variant-2 observations
constexpr int MAX_EDGES = MAX_NODES * 3 / 2;
constexpr int RNG_BUF = 256;

__device__ __forceinline__ int lane_id() { return threadIdx.x; }

__device__ __forceinline__ int readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t readlane_u(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    uint64_t b = __double_as_longlong(v);
    uint32_t lo = readlane_u((uint32_t)b, l), hi = readlane_u((uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l) {
    uint32_t lo = readlane_u((uint32_t)v, l), hi = readlane_u((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }

// 128-bit node sets (N <= 128): word v >> 6, bit v & 63
__device__ __forceinline__ bool bit128(const uint64_t* m, int v) { return (m[v >> 6] >> (v & 63)) & 1ull; }
__device__ __forceinline__ void set128(uint64_t* m, int v) { m[v >> 6] |= 1ull << (v & 63); }

__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#pragma unroll
    for (int m = 1; m < WAVE; m <<= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, m);
        hi |= (uint32_t)__shfl_xor((int)hi, m);
    }
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int m = 1; m < WAVE; m <<= 1) v += __shfl_xor(v, m);
    return v;
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
    uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

// In-place MT19937 generation of a 624-word block held in LDS, wave-parallel.
// Element i needs old[i], old[i+1] and either old[i+397] (i < 227) or new[i-227];
// processing 64-element chunks in order keeps every dependency resolved because
// 227 > 64. Loads of a chunk complete (barrier) before its stores.
__device__ __forceinline__ void mt_twist_lds(uint32_t* k) {
    const int l = lane_id();
    for (int s = 0; s < MT_N; s += WAVE) {
        int i = s + l;
        uint32_t a = 0, b = 0, m = 0;
        if (i < MT_N) {
            a = k[i];
            b = k[i == MT_N - 1 ? 0 : i + 1];
            m = k[i < MT_N - MT_M ? i + MT_M : i - (MT_N - MT_M)];
        }
        __syncthreads();
        if (i < MT_N) k[i] = mt_mix(a, b, m);
        __syncthreads();
    }
}

// numpy's init_genrand (RandomState.seed(int)); serial chain, written by lane 0. n < MT_N: only the
// first n state words (a partial block: LocalRng::seed_partial).
__device__ __forceinline__ void mt_seed_lds(uint32_t* k, uint32_t seed, int n = MT_N) {
    if (lane_id() == 0) {
        uint32_t v = seed;
        k[0] = v;
        for (int i = 1; i < n; i++) {
            v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
            k[i] = v;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t mask_for(uint32_t rng) {
    uint32_t m = rng;
    m |= m >> 1; m |= m >> 2; m |= m >> 4; m |= m >> 8; m |= m >> 16;
    return m;
}

// Per-env main stream: a ring of two 624-word blocks in HBM (block `cur`, position
// `pos`; block 1-cur holds the next generation when has_next). Tempered words are
// prefetched into LDS so that uniform sequential consumers read them at LDS latency.
struct MainRng {
    uint32_t* g;      // env's [2][624] key blocks (global)
    uint32_t* buf;    // LDS [RNG_BUF] tempered words
    uint32_t* tmp;    // LDS [624] twist scratch
    int cur, pos, has_next;
    int n, k;         // words in buf, consumed

    __device__ void twist_next() {
        const int l = lane_id();
        const uint32_t* src = g + cur * MT_N;
        for (int i = l; i < MT_N; i += WAVE) tmp[i] = src[i];
        __syncthreads();
        mt_twist_lds(tmp);
        uint32_t* dst = g + (1 - cur) * MT_N;
        for (int i = l; i < MT_N; i += WAVE) dst[i] = tmp[i];
        __syncthreads();
        has_next = 1;
    }
    // pos == 624 without a generated next block means "twist before the next draw"
    // (a freshly seeded numpy stream); only a generated next block can be entered.
    __device__ void commit() {
        pos += k;
        n = 0;
        k = 0;
        if (pos >= MT_N && has_next) {
            pos -= MT_N;
            cur = 1 - cur;
            has_next = 0;
        }
    }
    // wave-cooperative; uniform control flow only
    __device__ void prefetch(int want) {
        commit();
        if (want > RNG_BUF) want = RNG_BUF;
        if (pos + want > MT_N && !has_next) twist_next();
        int avail = (MT_N - pos) + (has_next ? MT_N : 0);
        if (want > avail) want = avail;
        const int l = lane_id();
        for (int i = l; i < want; i += WAVE) {
            int o = pos + i;
            uint32_t w = o < MT_N ? g[cur * MT_N + o] : g[(1 - cur) * MT_N + (o - MT_N)];
            buf[i] = mt_temper(w);
        }
        __syncthreads();
        n = want;
    }
    __device__ __forceinline__ uint32_t next32() {
        if (k >= n) prefetch(RNG_BUF);
        return buf[k++];
    }
    __device__ __forceinline__ int64_t randint(int64_t high) {  // legacy masked rejection
        uint32_t rng = (uint32_t)(high - 1);
        if (rng == 0) return 0;
        uint32_t m = mask_for(rng), v;
        // acceptance >= 1/2 per draw: 4096 rejections in a row means a broken stream
        for (int guard = 0; (v = (next32() & m)) > rng; guard++)
            if (guard > 4096) return 0;
        return (int64_t)v;
    }
    __device__ __forceinline__ double random() {
        int32_t a = (int32_t)(next32() >> 5), b = (int32_t)(next32() >> 6);
        return (a * 67108864.0 + b) / 9007199254740992.0;
    }
};

// Stream held entirely in LDS (fresh topology stream, network.py:242).
struct LocalRng {
    uint32_t* key;
    int pos;
    int lim = MT_N;     // generated words valid in key[0, lim) (< MT_N after seed_partial)
    uint32_t sd = 0;    // the seed (to complete a partial block)
    __device__ void seed(uint32_t s) {
        mt_seed_lds(key, s);
        pos = MT_N;
        lim = MT_N;
        sd = s;
    }
    // Seed and generate only the first w (<= MT_N - MT_M) words of the first block: word i < 227 of a
    // generation needs state words i, i + 1 and i + 397 only, so the serial seeding stops at 397 + w
    // instead of 624 (a topology attempt reads 4N + 1 words; 22 % of the chain at N = 20). A read past
    // word w rebuilds the whole block (same words).
    __device__ void seed_partial(uint32_t s, int w) {
        mt_seed_lds(key, s, MT_M + w);
        const int l = lane_id();
        for (int c = 0; c < w; c += WAVE) {  // in place, chunk by chunk like mt_twist_lds
            const int i = c + l;
            uint32_t a = 0, b = 0, m = 0;
            if (i < w) {
                a = key[i];
                b = key[i + 1];
                m = key[i + MT_M];
            }
            __syncthreads();
            if (i < w) key[i] = mt_mix(a, b, m);
            __syncthreads();
        }
        pos = 0;
        lim = w;
        sd = s;
    }
    __device__ __forceinline__ uint32_t next32() {
        if (pos == MT_N) {
            mt_twist_lds(key);
            pos = 0;
        }
        if (pos >= lim) {  // past a partial block: generate it completely
            mt_seed_lds(key, sd);
            mt_twist_lds(key);
            lim = MT_N;
        }
        return mt_temper(key[pos++]);
    }
    __device__ __forceinline__ int64_t randint(int64_t high) {
        uint32_t rng = (uint32_t)(high - 1);
        if (rng == 0) return 0;
        uint32_t m = mask_for(rng), v;
        for (int guard = 0; (v = (next32() & m)) > rng; guard++)
            if (guard > 4096) return 0;
        return (int64_t)v;
    }
};

}  // namespace gm

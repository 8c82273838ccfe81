// gm_env.hip — batched routing environment (reference src/env/routing.py,
// src/env/network.py) as HIP kernels for gfx950, plus its C ABI.
//
// Layout in HBM (library-owned, SoA per field, env-major):
//   packets  int32 [n_env][A] now/target/edge/time/ttl/start/spw/steps,
//            f64 size[n_env][A], u64 visited[n_env][A][2], u8 amask[n_env][A][4]
//   loads    f64 [n_env][E]            (E = 3N/2)
//   topology int32 nbr/nbr_edge [n_env][N][3] (ascending neighbour id),
//            int32 edge_a/edge_b/edge_len [n_env][E], int16 apsp [n_env][N][N]
//   rng      u32 [n_env][2][624] + cur/pos/has_next (numpy legacy MT19937 ring)
// One 64-lane wavefront per env: lane a owns packet a, lane e owns edge e (and
// e+64), so the order-dependent fp64 load updates are exact per-edge scans in
// packet-id order and every RNG draw happens in reference order.
//
// Compiled with -ffp-contract=off: the env is bit-exact against the reference.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/graph_marl_amd.h"
#include "gm_device.hpp"

using namespace gm;

namespace {
thread_local std::string g_err;
}

extern "C" const char* gm_last_error(void) { return g_err.c_str(); }
extern "C" int gm_version(void) { return 1; }

int gm_fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define GM_HIP(call)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return gm_fail(GM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct EnvDev {
    int n_env, N, A, E;
    int env_var, k;  // observation variant (routing.py:268-358) and variant-2 neighbour count
    int cong, amask_on, ttl, topo_mode, n_list, n_excl, seq_stride;
    int64_t fixed_seed;
    const int64_t* list;
    const int64_t* excl;
    int32_t *nbr, *nbr_edge, *edge_a, *edge_b, *edge_len;
    int16_t* apsp;
    int64_t* topo_seed;
    int32_t *topo_reps, *topo_ready, *seq_index;
    int32_t *now, *target, *edge, *time, *ttl_, *start, *spw, *steps;
    double* size;
    uint64_t* visited;
    uint8_t* amask;
    double* load;
    uint32_t* mt;
    int32_t *mt_cur, *mt_pos, *mt_has_next;
    int32_t* err;
};

struct gm_env {
    gm_env_config cfg;
    std::vector<int64_t> list, excl;
    EnvDev d;
    std::vector<void*> allocs;
    int device;
};

namespace {

// ---------------------------------------------------------------------------
// Shared per-block LDS image of one env
// ---------------------------------------------------------------------------
// NC = node capacity of the kernel instance (64 or 128, picked from N at launch so
// that N <= 64 keeps the small LDS footprint and occupancy)
template <int NC>
struct EnvLds {
    int32_t now[MAX_AGENTS], target[MAX_AGENTS], edge[MAX_AGENTS], time[MAX_AGENTS];
    double size[MAX_AGENTS];
    double load[NC * 3 / 2];
    uint8_t nbr[NC * 3], nbr_edge[NC * 3];
    uint8_t ea[NC * 3 / 2], eb[NC * 3 / 2], elen[NC * 3 / 2];
    uint64_t nbrmask[NC][2];
    int8_t kn[MAX_AGENTS][MAX_KNBR];  // variant 2: the first k packets on the same / an adjacent node
    float node_cnt[NC], node_load[NC];
    alignas(16) uint32_t rbuf[RNG_BUF];  // rbuf + rtmp (contiguous): also the observation staging image
    uint32_t rtmp[MT_N];
};
constexpr int STG_FLOATS = RNG_BUF + MT_N;  // >= one row of either observation at N = 128

template <class ES>
__device__ void load_topology_lds(const EnvDev& d, int env, ES& s) {
    const int l = lane_id();
    const int N = d.N, E = d.E;
    for (int i = l; i < N * 3; i += WAVE) {
        s.nbr[i] = (uint8_t)d.nbr[(size_t)env * N * 3 + i];
        s.nbr_edge[i] = (uint8_t)d.nbr_edge[(size_t)env * N * 3 + i];
    }
    for (int e = l; e < E; e += WAVE) {
        s.ea[e] = (uint8_t)d.edge_a[(size_t)env * E + e];
        s.eb[e] = (uint8_t)d.edge_b[(size_t)env * E + e];
        s.elen[e] = (uint8_t)d.edge_len[(size_t)env * E + e];
    }
    __syncthreads();
    for (int v = l; v < N; v += WAVE) {
        uint64_t m[2] = {0ull, 0ull};
        for (int k = 0; k < 3; k++) set128(m, s.nbr[v * 3 + k]);
        s.nbrmask[v][0] = m[0];
        s.nbrmask[v][1] = m[1];
    }
    __syncthreads();
}

template <class ES>
__device__ __forceinline__ MainRng open_rng(const EnvDev& d, int env, ES& s) {
    MainRng r;
    r.g = d.mt + (size_t)env * 2 * MT_N;
    r.buf = s.rbuf;
    r.tmp = s.rtmp;
    r.cur = d.mt_cur[env];
    r.pos = d.mt_pos[env];
    r.has_next = d.mt_has_next[env];
    r.n = 0;
    r.k = 0;
    return r;
}

__device__ __forceinline__ void close_rng(const EnvDev& d, int env, MainRng& r) {
    r.commit();
    if (lane_id() == 0) {
        d.mt_cur[env] = r.cur;
        d.mt_pos[env] = r.pos;
        d.mt_has_next[env] = r.has_next;
    }
}

// ---------------------------------------------------------------------------
// Observation emission (routing.py:187-358, 522-539), packet state in LDS.
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ int obs_dim_of(int N, int env_var, int k) {
    return 6 * N + 10 + (env_var == 2 ? 5 * k : 0) + (env_var == 3 ? N * N + N * (4 * N + 8) : 0);
}

// node observation entry (routing.py:187-235) from the per-node packet count / size sums
// (block k, offset q) of column r of the 3 neighbour blocks of N+2 columns (no division)
__device__ __forceinline__ void nbr_block(int r, int N, int& k, int& q) {
    k = (r >= N + 2) + (r >= 2 * (N + 2));
    q = r - k * (N + 2);
}

// value of neighbour-block column (k, q) of node v: onehot(nbr) | edge length | edge load
template <class ES>
__device__ __forceinline__ float nbr_block_value(const ES& s, int N, int v, int k, int q) {
    const int nb = s.nbr[v * 3 + k], ne = s.nbr_edge[v * 3 + k];
    return q < N ? (float)(nb == q) : (q == N ? (float)s.elen[ne] : (float)s.load[ne]);
}

template <class ES>
__device__ __forceinline__ float node_obs_value(const ES& s, int N, int j, int c) {
    if (c < N) return (float)(c == j);
    if (c == N) return s.node_cnt[j];
    if (c == N + 1) return s.node_load[j];
    int k, q;
    nbr_block(c - (N + 2), N, k, q);
    return nbr_block_value(s, N, j, k, q);
}


// Observation rows are one-hot blocks plus a few scalars: zero-fill (one flat lane-strided
// pass), then each lane writes the entries of its own row (no per-column branch chains).

template <class ES>
__device__ void emit_obs(const EnvDev& d, int env, ES& s, const gm_obs_buffers& o) {
    const int l = lane_id();
    const int N = d.N, A = d.A;
    if (o.node_obs || (o.obs && d.env_var == 3)) {
        // packets waiting at node j (not on an edge) and the sum of their sizes in id order
        for (int v = l; v < N; v += WAVE) {
            int cnt = 0;
            double tl = 0.0;
            for (int i = 0; i < A; i++) {
                if (s.now[i] == v && s.edge[i] == -1) {
                    cnt++;
                    tl += s.size[i];
                }
            }
            s.node_cnt[v] = (float)cnt;
            s.node_load[v] = (float)tl;
        }
        __syncthreads();
        if (o.node_obs) {
            // routing.py:187-235. Rows are mostly zeros: batches of rows are built in an LDS image
            // (zero-fill, then each lane writes the 12 nonzero-capable entries of its node) and
            // leave as full 16-byte stores of the env's contiguous N x (4N+8) block, so every HBM
            // byte is written once (a zero-fill + scatter in HBM costs partial-line rewrites)
            const int ND = 4 * N + 8;
            float* base = o.node_obs + (size_t)env * N * ND;
            float* stg = reinterpret_cast<float*>(s.rbuf);  // rbuf + rtmp: the RNG is closed here
            const int per = STG_FLOATS / ND;
            const bool vec = (reinterpret_cast<uintptr_t>(base) & 15) == 0;  // N*ND is a multiple of 4
            for (int v0 = 0; v0 < N; v0 += per) {
                const int nr = min(per, N - v0), nf = nr * ND;  // nf is a multiple of 4 (ND = 4N+8)
                for (int i = l; i < nf / 4; i += WAVE) reinterpret_cast<float4*>(stg)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
                __syncthreads();
                if (l < nr) {
                    const int v = v0 + l;
                    float* row = stg + l * ND;
                    row[v] = 1.f;
                    row[N] = s.node_cnt[v];
                    row[N + 1] = s.node_load[v];
#pragma unroll
                    for (int k = 0; k < 3; k++) {
                        float* blk = row + N + 2 + k * (N + 2);
                        const int ne = s.nbr_edge[v * 3 + k];
                        blk[s.nbr[v * 3 + k]] = 1.f;
                        blk[N] = (float)s.elen[ne];
                        blk[N + 1] = (float)s.load[ne];
                    }
                }
                __syncthreads();
                float* dst = base + (size_t)v0 * ND;
                if (vec) {
                    for (int i = l; i < nf / 4; i += WAVE)
                        reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(stg)[i];
                } else {
                    for (int i = l; i < nf; i += WAVE) dst[i] = stg[i];
                }
                __syncthreads();
            }
        }
    }
    if (o.obs && d.env_var == 2) {
        // routing.py:317-342: packets j != a in id order on a's node or a neighbour; the
        // first k contribute (now, target, edge, size, a) — the reference appends its own id
        if (l < A) {
            const int now = s.now[l];
            int cnt = 0;
            for (int j = 0; j < A && cnt < d.k; j++) {
                if (j == l) continue;
                const int nj = s.now[j];
                if (nj == now || bit128(s.nbrmask[now], nj)) s.kn[l][cnt++] = (int8_t)j;
            }
            for (int q = cnt; q < d.k; q++) s.kn[l][q] = -1;
        }
        __syncthreads();
    }
    if (o.obs || o.obs_gemm) {
        // routing.py:269-315. The INDEPENDENT part of a row has at most 16 nonzero entries:
        // zero-fill columns [0, 6N+10) of all A rows, then lane a writes packet a's entries.
        // obs NULL with obs_gemm set: only the GEMM-ready copy is written (gm_obs_from_gemm
        // rebuilds the agent rows from it on demand)
        const int D1 = 6 * N + 10, D = obs_dim_of(N, d.env_var, d.k);
        const size_t ld = o.obs_row_stride;
        float* base = o.obs ? o.obs + (size_t)env * A * ld : nullptr;
        // routing.py:269-315. The INDEPENDENT part of a row has at most 16 nonzero entries:
        // batches of rows are built in the LDS image (row stride SR = D1 rounded up to 4 floats),
        // then copied out row by row as 16-byte stores (the last 2 columns of D1 = 4q + 2 as a
        // pair), each HBM byte written once
        float* stg = reinterpret_cast<float*>(s.rbuf);
        const int SR = (D1 + 3) & ~3, Q = D1 / 4, T = D1 - 4 * Q, per = STG_FLOATS / SR;
        const bool vec = (ld & 3) == 0 && (reinterpret_cast<uintptr_t>(base) & 15) == 0;
        for (int a0 = 0; a0 < A; a0 += per) {
            const int nr = min(per, A - a0);
            for (int i = l; i < nr * SR / 4; i += WAVE) reinterpret_cast<float4*>(stg)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
            __syncthreads();
            if (l < nr) {
                const int a = a0 + l;
                float* row = stg + l * SR;
                const int now = s.now[a], e = s.edge[a];
                row[now] = 1.f;
                row[N + s.target[a]] = 1.f;
                row[2 * N] = (float)(e != -1);
                if (e >= 0) row[2 * N + 1 + (s.ea[e] ^ s.eb[e] ^ now)] = 1.f;
                row[3 * N + 1] = (float)s.time[a];
                row[3 * N + 2] = (float)s.size[a];
                row[3 * N + 3] = (float)a;
#pragma unroll
                for (int k = 0; k < 3; k++) {
                    float* blk = row + 3 * N + 4 + k * (N + 2);
                    const int ne = s.nbr_edge[now * 3 + k];
                    blk[s.nbr[now * 3 + k]] = 1.f;
                    blk[N] = (float)s.elen[ne];
                    blk[N + 1] = (float)s.load[ne];
                }
            }
            __syncthreads();
            if (!base) {
            } else if (vec) {
                const int Qr = Q + (T ? 1 : 0);  // 16-B chunks per row, the last one partial (T = 2)
                for (int i = l; i < nr * Qr; i += WAVE) {
                    const int r = i / Qr, q = i - r * Qr;
                    const float4 v = *reinterpret_cast<const float4*>(stg + r * SR + 4 * q);
                    float* dst = base + (size_t)(a0 + r) * ld + 4 * q;
                    if (q < Q) {
                        *reinterpret_cast<float4*>(dst) = v;
                    } else if (T == 2) {  // D1 = 6N + 10 with N even
                        *reinterpret_cast<float2*>(dst) = make_float2(v.x, v.y);
                    } else {
                        for (int c = 0; c < T; c++) dst[c] = stg[r * SR + 4 * q + c];
                    }
                }
            } else {
                for (int i = l; i < nr * D1; i += WAVE) {
                    const int r = i / D1, c = i - r * D1;
                    base[(size_t)(a0 + r) * ld + c] = stg[r * SR + c];
                }
            }
            if (o.obs_gemm) {  // the GEMM copy without columns N-1 and 2N (host-checked: var 1, 16-B rows)
                const int Qg = (D1 - 2) / 4;  // 6N+8 = 4 Qg (N even)
                float* gb = o.obs_gemm + ((size_t)env * A + a0) * o.obs_gemm_stride;
                for (int i = l; i < nr * Qg; i += WAVE) {
                    const int r = i / Qg, q = i - r * Qg;
                    float v[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int c = 4 * q + j;
                        v[j] = stg[r * SR + (c < N - 1 ? c : (c < 2 * N - 1 ? c + 1 : c + 2))];
                    }
                    *reinterpret_cast<float4*>(gb + (size_t)r * o.obs_gemm_stride + 4 * q) =
                        make_float4(v[0], v[1], v[2], v[3]);
                }
            }
            __syncthreads();
        }
        if (base && D > D1) {  // variant columns (2: k neighbour slots, 3: global), lane-strided per row
            for (int a = 0; a < A; a++) {
                float* row = base + (size_t)a * ld;
                for (int c = D1 + l; c < D; c += WAVE) {
                    const int g = c - D1;
                    float v;
                    if (d.env_var == 2) {  // k neighbour slots of 5, -1 placeholders
                        const int slot = g / 5, f = g - slot * 5, j = s.kn[a][slot];
                        v = j < 0 ? -1.0f
                                  : f == 0 ? (float)s.now[j]
                                  : f == 1 ? (float)s.target[j]
                                  : f == 2 ? (float)s.edge[j]
                                  : f == 3 ? (float)s.size[j] : (float)a;
                    } else if (g < N * N) {  // variant 3: I + A flattened, then node obs
                        const int r = g / N, q = g - r * N;
                        v = (float)(r == q || bit128(s.nbrmask[r], q));
                    } else {
                        const int ND = 4 * N + 8, h = g - N * N, j = h / ND;
                        v = node_obs_value(s, N, j, h - j * ND);
                    }
                    row[c] = v;
                }
            }
        }
    }
    if (o.agent_node && l < A) o.agent_node[(size_t)env * A + l] = s.now[l];
    if (o.agent_adj) {
        int8_t* base = o.agent_adj + (size_t)env * A * A;
        for (int idx = l; idx < A * A; idx += WAVE) {
            int i = idx / A, j = idx - i * A;
            int ni = s.now[i], nj = s.now[j];
            base[idx] = (int8_t)(i == j || ni == nj || bit128(s.nbrmask[ni], nj));
        }
    }
}

template <class ES>
__device__ void load_packets_lds(const EnvDev& d, int env, ES& s) {
    const int l = lane_id();
    if (l < d.A) {
        size_t p = (size_t)env * d.A + l;
        s.now[l] = d.now[p];
        s.target[l] = d.target[p];
        s.edge[l] = d.edge[p];
        s.time[l] = d.time[p];
        s.size[l] = d.size[p];
    }
    for (int e = l; e < d.E; e += WAVE) s.load[e] = d.load[(size_t)env * d.E + e];
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Topology generation (network.py:122-272), one wave per env, state in LDS.
// ---------------------------------------------------------------------------
template <int NC>
struct TopoLds {
    static constexpr int NCAP = NC;
    double x[NC], y[NC], d2[NC];
    uint32_t tkey[MT_N];
    int32_t deg[NC];
    uint64_t adj[NC][2];
    int32_t node_edges[NC * 3];
    int32_t ea[NC * 3 / 2], eb[NC * 3 / 2], elen[NC * 3 / 2];
    int32_t n_edges;
    int32_t cand_at_rank[NC];
    uint8_t ok_at_rank[NC];
};

__device__ __forceinline__ bool is_excluded(const EnvDev& d, int64_t sd) {
    int lo = 0, hi = d.n_excl - 1;
    while (lo <= hi) {
        int m = (lo + hi) >> 1;
        int64_t v = d.excl[m];
        if (v == sd) return true;
        if (v < sd) lo = m + 1;
        else hi = m - 1;
    }
    return false;
}

template <class R>
__device__ int64_t draw_topology_seed(const EnvDev& d, R& r) {  // network.py:230-232, 252-254
    int64_t sd = r.randint(2147483647LL);
    for (int guard = 0; d.n_excl > 0 && is_excluded(d, sd) && guard < 4096; guard++) sd = r.randint(2147483647LL);
    return sd;
}

// one min step of a wave reduction over 64-bit keys: the partner lane by a DPP pattern (no LDS round trip)
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_min_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    return o < v ? o : v;
}
// the smallest key over the lanes with `in` (uniform result); ~0 when no lane has `in`. Call it with every
// lane active (outside any lane condition). Inside each 16-lane row by DPP (quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror: every lane ends with its row's minimum), then the four rows by readlane:
// ~8x shorter than a 6-round shuffle butterfly, whose LDS-path bpermutes dominated an attempt's rows
__device__ __forceinline__ uint64_t argmin_key(uint64_t key, bool in) {
    uint64_t v = in ? key : ~0ull;
    v = dpp_min_u64<0xB1>(v);
    v = dpp_min_u64<0x4E>(v);
    v = dpp_min_u64<0x141>(v);
    v = dpp_min_u64<0x140>(v);
    const uint64_t r0 = readlane_u64(v, 0), r1 = readlane_u64(v, 16), r2 = readlane_u64(v, 32), r3 = readlane_u64(v, 48);
    const uint64_t a = r0 < r1 ? r0 : r1, b = r2 < r3 ? r2 : r3;
    return a < b ? a : b;
}

// One _create_random_topology attempt (network.py:122-195) for N <= 64, lane v = node v, the whole
// state in registers (round 5; the LDS form below took ~100 k cycles per attempt at N = 20, and a reset
// lasts as long as its worst env's attempt chain: ~17 attempts at 4096 envs). Row i's candidates are
// taken in the reference's stable sort order of (squared distance, index) without sorting: the first
// element (sorted index 0, normally i itself) and then the takeable nodes one by one as wave minima of
// the distance bits (non-negative doubles order like their bit patterns) with the lowest index among
// equal keys. Takeability (degree < 3, not yet linked to i) is evaluated at the start of the row: no
// candidate's state changes before it is visited, and the row stops when i has 3 neighbours, so this
// equals the reference's check at visit time. Edge records go to LDS (written by the candidate's lane,
// read after the caller's barrier); degrees, edge slots and adjacency bits stay in the owning lane's
// registers and are written to LDS at the end for topology_finish.
template <class TS>
__device__ bool topology_attempt_reg(const EnvDev& d, TS& t, LocalRng& tr) {
    const int l = lane_id();
    const int N = d.N;
    if (tr.pos == MT_N) {
        mt_twist_lds(tr.key);
        tr.pos = 0;
    }
    const bool live = l < N;
    double x = 0.0, y = 0.0;
    if (live) {
        uint32_t w0 = mt_temper(tr.key[tr.pos + 4 * l]), w1 = mt_temper(tr.key[tr.pos + 4 * l + 1]);
        uint32_t w2 = mt_temper(tr.key[tr.pos + 4 * l + 2]), w3 = mt_temper(tr.key[tr.pos + 4 * l + 3]);
        x = ((int32_t)(w0 >> 5) * 67108864.0 + (int32_t)(w1 >> 6)) / 9007199254740992.0;
        y = ((int32_t)(w2 >> 5) * 67108864.0 + (int32_t)(w3 >> 6)) / 9007199254740992.0;
    }
    tr.pos += 4 * N;
    int deg = 0, ne0 = 0, ne1 = 0, ne2 = 0, n_edges = 0;
    uint64_t adj = 0ull;
    for (int i = 0; i < N; i++) {
        const int need = 3 - readlane(deg, i);
        if (need <= 0) continue;  // the reference's loop breaks at once
        const double xi = readlane_f64(x, i), yi = readlane_f64(y, i);
        const double dx = x - xi, dy = y - yi;
        const double a = dx * dx, b = dy * dy;
        const double d2 = a + b;  // >= +0: its IEEE bits order like the values
        const uint64_t key = live ? (uint64_t)__double_as_longlong(d2) : ~0ull;
        // edge length of every node as a candidate of row i (network.py:173), all lanes at once
        const double s10 = sqrt(d2) * 10.0;
        const int32_t len = ((int32_t)s10) / 2 + 1;
        // sorted index 0 (skipped: normally i itself) = the first (key, index) of all nodes; then the
        // candidates in sort order = successive (key, index) minima over the takeable nodes (the row's
        // start-of-row state, a lane mask), each a wave min + ballot (ties: the lowest index, as the
        // stable sort keeps them)
        const uint64_t kmin = argmin_key(key, live);  // outside any condition: every lane takes part
        const uint64_t r0m = ballot(live && key == kmin);
        uint64_t cands = ballot(live && deg < 3 && !((adj >> i) & 1ull)) & ~(r0m & (0ull - r0m));
        for (int j = 0; j < need && cands; j++) {
            const bool in = (cands >> l) & 1ull;
            const uint64_t cmin = argmin_key(key, in);
            const uint64_t hit = ballot(in && key == cmin);
            const int c = __builtin_ctzll(hit);
            cands &= ~(1ull << c);
            const int e = n_edges++;
            if (l == c) {  // the candidate's lane records the edge (one writer)
                t.ea[e] = i < c ? i : c;
                t.eb[e] = i < c ? c : i;
                t.elen[e] = len;
            }
            // candidate first, then i (network.py:180-181)
            if (l == c) {
                ne0 = deg == 0 ? e : ne0;
                ne1 = deg == 1 ? e : ne1;
                ne2 = deg == 2 ? e : ne2;
                deg += 1;
                adj |= 1ull << i;
            }
            if (l == i) {
                ne0 = deg == 0 ? e : ne0;
                ne1 = deg == 1 ? e : ne1;
                ne2 = deg == 2 ? e : ne2;
                deg += 1;
                adj |= 1ull << c;
            }
        }
    }
    if (live) {
        t.node_edges[l * 3 + 0] = ne0;
        t.node_edges[l * 3 + 1] = ne1;
        t.node_edges[l * 3 + 2] = ne2;
        t.deg[l] = deg;
        t.adj[l][0] = adj;
        t.adj[l][1] = 0ull;
    }
    if (l == 0) t.n_edges = n_edges;
    // validity (network.py:197-213): all degrees 3 and connected
    if (ballot(live && deg != 3)) return false;
    const uint64_t full = N == 64 ? ~0ull : ((1ull << N) - 1);
    uint64_t reach = 1ull, prev = 0ull;
    while (reach != prev) {
        prev = reach;
        reach |= wave_or_u64(((prev >> l) & 1ull) && live ? adj : 0ull);
    }
    return reach == full;
}

// One _create_random_topology attempt from the LDS stream t.tkey (fresh after seeding).
// Node-indexed work runs in lanes v = l and v = l + 64 (N <= 128); N <= 64: topology_attempt_reg.
template <class TS>
__device__ bool topology_attempt(const EnvDev& d, TS& t, LocalRng& tr) {
    if constexpr (TS::NCAP <= 64) return topology_attempt_reg(d, t, tr);
    const int l = lane_id();
    const int N = d.N;
    // positions: node i draws x then y (network.py:134-138) = tempered words 4i..4i+3
    // (4N <= 512 words: one fresh 624-word block)
    if (tr.pos == MT_N) {
        mt_twist_lds(tr.key);
        tr.pos = 0;
    }
    for (int v = l; v < N; v += WAVE) {
        uint32_t w0 = mt_temper(tr.key[tr.pos + 4 * v]), w1 = mt_temper(tr.key[tr.pos + 4 * v + 1]);
        uint32_t w2 = mt_temper(tr.key[tr.pos + 4 * v + 2]), w3 = mt_temper(tr.key[tr.pos + 4 * v + 3]);
        t.x[v] = ((int32_t)(w0 >> 5) * 67108864.0 + (int32_t)(w1 >> 6)) / 9007199254740992.0;
        t.y[v] = ((int32_t)(w2 >> 5) * 67108864.0 + (int32_t)(w3 >> 6)) / 9007199254740992.0;
        t.deg[v] = 0;
        t.adj[v][0] = 0;
        t.adj[v][1] = 0;
    }
    tr.pos += 4 * N;
    if (l == 0) t.n_edges = 0;
    __syncthreads();
    for (int i = 0; i < N; i++) {
        // squared distances of row i (network.py:143-150) and stable ranks (153)
        double my[2] = {0.0, 0.0};
        for (int h = 0; h < 2; h++) {
            const int v = l + h * WAVE;
            if (v < N) {
                double dx = t.x[v] - t.x[i], dy = t.y[v] - t.y[i];
                double a = dx * dx, b = dy * dy;
                my[h] = a + b;
                t.d2[v] = my[h];
            }
        }
        __syncthreads();
        int rank[2] = {0, 0};
        for (int h = 0; h < 2; h++) {
            const int v = l + h * WAVE;
            if (v < N) {
                for (int k = 0; k < N; k++) {
                    double dk = t.d2[k];
                    rank[h] += (dk < my[h]) || (dk == my[h] && k < v);
                }
            }
        }
        const int need = 3 - t.deg[i];
        if (need > 0) {
            // candidate at sorted position r >= 1 is taken iff its degree < 3 and it is
            // not already linked to i (network.py:157-170), first `need` in rank order
            for (int h = 0; h < 2; h++) {
                const int v = l + h * WAVE;
                if (v < N) {
                    bool ok = rank[h] >= 1 && t.deg[v] < 3 && !bit128(t.adj[v], i);
                    t.ok_at_rank[rank[h]] = (uint8_t)ok;
                    t.cand_at_rank[rank[h]] = v;
                }
            }
            __syncthreads();
            uint64_t okm0 = ballot(l < N && t.ok_at_rank[l]);
            uint64_t okm1 = ballot(l + WAVE < N && t.ok_at_rank[l + WAVE]);
            int take = 0;
            while ((okm0 | okm1) && take < need) {
                int r;
                if (okm0) {
                    r = __builtin_ctzll(okm0);
                    okm0 &= okm0 - 1;
                } else {
                    r = WAVE + __builtin_ctzll(okm1);
                    okm1 &= okm1 - 1;
                }
                take++;
                int c = t.cand_at_rank[r];
                double dc = t.d2[c];
                double sq = sqrt(dc);
                double s10 = sq * 10.0;
                int32_t len = ((int32_t)s10) / 2 + 1;  // network.py:173
                if (l == 0) {
                    int e = t.n_edges;
                    t.ea[e] = i < c ? i : c;
                    t.eb[e] = i < c ? c : i;
                    t.elen[e] = len;
                    t.node_edges[c * 3 + t.deg[c]] = e;  // candidate first (180-181)
                    t.deg[c] += 1;
                    t.node_edges[i * 3 + t.deg[i]] = e;
                    t.deg[i] += 1;
                    set128(t.adj[c], i);
                    set128(t.adj[i], c);
                    t.n_edges = e + 1;
                }
                __syncthreads();
            }
        }
        __syncthreads();
    }
    // validity (network.py:197-213): all degrees 3 and connected
    bool deg_ok = !(ballot(l < N && t.deg[l] != 3) | ballot(l + WAVE < N && t.deg[l + WAVE] != 3));
    if (!deg_ok) return false;
    uint64_t full0 = N >= 64 ? ~0ull : ((1ull << N) - 1);
    uint64_t full1 = N <= 64 ? 0ull : (N == 128 ? ~0ull : ((1ull << (N - 64)) - 1));
    uint64_t reach[2] = {1ull, 0ull}, prev[2] = {0ull, 0ull};
    while (reach[0] != prev[0] || reach[1] != prev[1]) {
        prev[0] = reach[0];
        prev[1] = reach[1];
        uint64_t c0 = 0, c1 = 0;
        for (int h = 0; h < 2; h++) {
            const int v = l + h * WAVE;
            if (v < N && bit128(prev, v)) {
                c0 |= t.adj[v][0];
                c1 |= t.adj[v][1];
            }
        }
        reach[0] |= wave_or_u64(c0);
        reach[1] |= wave_or_u64(c1);
    }
    return reach[0] == full0 && reach[1] == full1;
}

// Floyd-Warshall for N <= NC <= 64 with the distance matrix in registers: lane j holds column j
// (dist[i][j], i < NC: static register indices); pivot k broadcasts column k through LDS (col, NC int32)
// and dist[k][j] = dist[j][k] (symmetric) is entry j of that column. Integer min-plus: the same result as
// the LDS form in any order. Pads (i or j >= N) hold INF and never shorten a path.
template <int NC, class TS>
__device__ void apsp_reg(const EnvDev& d, int env, const TS& t, int32_t* col) {
    static_assert(NC <= 64 && NC % 4 == 0, "register APSP needs NC <= 64");
    const int l = lane_id();
    const int N = d.N;
    constexpr int INF = 1 << 20;
    // column j: 0 on the diagonal, the edge lengths at j's three neighbours (a valid topology is simple
    // and 3-regular), INF elsewhere
    int nb[3] = {-1, -1, -1}, ln[3] = {0, 0, 0};
    if (l < N) {
#pragma unroll
        for (int q = 0; q < 3; q++) {
            const int e = t.node_edges[l * 3 + q];
            nb[q] = t.ea[e] ^ t.eb[e] ^ l;
            ln[q] = t.elen[e];
        }
    }
    int dc[NC];
#pragma unroll
    for (int i = 0; i < NC; i++)
        dc[i] = (i == l && l < N) ? 0 : i == nb[0] ? ln[0] : i == nb[1] ? ln[1] : i == nb[2] ? ln[2] : INF;
    for (int k = 0; k < N; k++) {
        int32_t* ck = col + (k & 1) * NC;  // double-buffered: one barrier per pivot
        if (l == k) {
#pragma unroll
            for (int i = 0; i < NC; i += 4) *reinterpret_cast<int4*>(ck + i) = make_int4(dc[i], dc[i + 1], dc[i + 2], dc[i + 3]);
        }
        __syncthreads();
        const int dkj = l < NC ? ck[l] : INF;
#pragma unroll
        for (int i = 0; i < NC; i += 4) {
            const int4 v = *reinterpret_cast<const int4*>(ck + i);
            dc[i] = min(dc[i], v.x + dkj);
            dc[i + 1] = min(dc[i + 1], v.y + dkj);
            dc[i + 2] = min(dc[i + 2], v.z + dkj);
            dc[i + 3] = min(dc[i + 3], v.w + dkj);
        }
    }
    if (l < N) {
#pragma unroll
        for (int i = 0; i < NC; i++)
            if (i < N) d.apsp[((size_t)env * N + i) * N + l] = (int16_t)dc[i];
    }
}

template <class TS>
__device__ void topology_finish(const EnvDev& d, int env, TS& t, int16_t* dist, int64_t seed, int reps) {
    const int l = lane_id();
    const int N = d.N, E = d.E;
    // per-node edges sorted by neighbour id (network.py:191-195)
    for (int v = l; v < N; v += WAVE) {
        int ee[3], nb[3];
        for (int k = 0; k < 3; k++) {
            ee[k] = t.node_edges[v * 3 + k];
            nb[k] = t.ea[ee[k]] ^ t.eb[ee[k]] ^ v;
        }
        for (int a = 1; a < 3; a++)
            for (int b = a; b > 0 && nb[b - 1] > nb[b]; b--) {
                int tn = nb[b]; nb[b] = nb[b - 1]; nb[b - 1] = tn;
                int te = ee[b]; ee[b] = ee[b - 1]; ee[b - 1] = te;
            }
        for (int k = 0; k < 3; k++) {
            d.nbr[((size_t)env * N + v) * 3 + k] = nb[k];
            d.nbr_edge[((size_t)env * N + v) * 3 + k] = ee[k];
        }
    }
    for (int e = l; e < E; e += WAVE) {
        d.edge_a[(size_t)env * E + e] = t.ea[e];
        d.edge_b[(size_t)env * E + e] = t.eb[e];
        d.edge_len[(size_t)env * E + e] = t.elen[e];
    }
    // all-pairs shortest path weights (network.py:274-290) by Floyd-Warshall
    if constexpr (TS::NCAP <= 64) {
        apsp_reg<TS::NCAP>(d, env, t, reinterpret_cast<int32_t*>(dist));
    } else {
    const int16_t INF = 0x3fff;
    for (int idx = l; idx < N * N; idx += WAVE) dist[idx] = (idx / N == idx % N) ? 0 : INF;
    __syncthreads();
    for (int e = l; e < E; e += WAVE) {
        int a = t.ea[e], b = t.eb[e];
        dist[a * N + b] = (int16_t)t.elen[e];
        dist[b * N + a] = (int16_t)t.elen[e];
    }
    __syncthreads();
    for (int k = 0; k < N; k++) {
        for (int idx = l; idx < N * N; idx += WAVE) {
            int i = idx / N, j = idx - i * N;
            int v = dist[i * N + k] + dist[k * N + j];
            if (v < dist[idx]) dist[idx] = (int16_t)v;
        }
        __syncthreads();
    }
    for (int idx = l; idx < N * N; idx += WAVE) d.apsp[(size_t)env * N * N + idx] = dist[idx];
    }
    if (l == 0) {
        d.topo_seed[env] = seed;
        d.topo_reps[env] = reps;
        d.topo_ready[env] = 1;
    }
}

// network.py:242-258: fresh stream per topology seed, reseed on invalid topology
template <class TS>
__device__ void generate_topology(const EnvDev& d, int env, TS& t, int16_t* dist, int64_t seed,
                                  bool allow_retry) {
    LocalRng tr;
    tr.key = t.tkey;
    // an attempt reads 4N position words and, when invalid, the next seed (one more word per rare
    // rejection): partial blocks while those fit the first MT_N - MT_M words
    const int w = 4 * d.N + 2;
    const bool part = w <= MT_N - MT_M;
    auto reseed = [&](int64_t sd) {
        if (part)
            tr.seed_partial((uint32_t)sd, w);
        else
            tr.seed((uint32_t)sd);
    };
    reseed(seed);
    int reps = 0;
    for (;;) {
        bool ok = topology_attempt(d, t, tr);
        reps++;
        if (ok) break;
        if (!allow_retry || reps > 100000) {
            if (lane_id() == 0) atomicExch(d.err, GM_ERR_TOPOLOGY);
            break;
        }
        seed = draw_topology_seed(d, tr);
        reseed(seed);
    }
    __syncthreads();
    topology_finish(d, env, t, dist, seed, reps);
    __syncthreads();
}

template <int NC>
struct ResetLds {
    EnvLds<NC> env;
    TopoLds<NC> topo;
    alignas(16) int16_t dist[NC * NC];  // Floyd-Warshall APSP (NC <= 64: the pivot column buffer)
};

// src/env/routing.py:160-178 (+ network.py:366-371): new topology (per mode), zero
// loads, respawn every packet in id order (reset_packet, routing.py:119-144).
template <int NC>
__global__ __launch_bounds__(64) void k_env_reset(EnvDev d, const uint8_t* mask, gm_obs_buffers o) {
    const int env = blockIdx.x;
    if (mask && !mask[env]) return;
    const int l = lane_id();
    __shared__ ResetLds<NC> S;
    EnvLds<NC>& s = S.env;
    MainRng r = open_rng(d, env, s);
    const int N = d.N, A = d.A;

    int64_t seed = -1;
    bool gen = true;
    if (d.topo_mode == GM_TOPO_FIXED) {
        gen = d.topo_ready[env] == 0;  // same topology every reset; no draw
        seed = d.fixed_seed;
    } else if (d.topo_mode == GM_TOPO_RANDOM) {
        seed = draw_topology_seed(d, r);
    } else if (d.topo_mode == GM_TOPO_LIST) {
        seed = d.list[r.randint(d.n_list)];  // np.random.choice(seed_list)
    } else {
        int idx = 0;
        if (d.n_list > 1) {
            idx = d.seq_index[env];
            __syncthreads();
            if (l == 0) d.seq_index[env] = (idx + d.seq_stride) % d.n_list;
        }
        seed = d.list[idx];
    }
    if (gen) generate_topology(d, env, S.topo, S.dist, seed, d.topo_mode == GM_TOPO_RANDOM);
    __syncthreads();

    // packets
    int p_now = 0, p_target = 0;
    double p_size = 0.0;
    for (int i = 0; i < A; i++) {
        int st = (int)r.randint(N);
        int tg = (int)r.randint(N);
        double sz = r.random();
        if (l == i) {
            p_now = st;
            p_target = tg;
            p_size = sz;
        }
    }
    close_rng(d, env, r);
    if (l < A) {
        size_t p = (size_t)env * A + l;
        d.now[p] = p_now;
        d.target[p] = p_target;
        d.start[p] = p_now;
        d.size[p] = p_size;
        d.edge[p] = -1;
        d.time[p] = 0;
        d.ttl_[p] = d.ttl;
        d.steps[p] = 0;
        d.spw[p] = d.apsp[((size_t)env * N + p_now) * N + p_target];
        d.visited[p * 2 + 0] = p_now < 64 ? (1ull << p_now) : 0ull;
        d.visited[p * 2 + 1] = p_now >= 64 ? (1ull << (p_now - 64)) : 0ull;
        uint32_t m = d.amask_on ? (uint32_t)(p_now != p_target) : 0u;
        reinterpret_cast<uint32_t*>(d.amask)[p] = m;
        s.now[l] = p_now;
        s.target[l] = p_target;
        s.edge[l] = -1;
        s.time[l] = 0;
        s.size[l] = p_size;
    }
    for (int e = l; e < d.E; e += WAVE) {
        d.load[(size_t)env * d.E + e] = 0.0;
        s.load[e] = 0.0;
    }
    __syncthreads();
    if (o.obs || o.obs_gemm || o.node_obs || o.agent_node || o.agent_adj) {
        load_topology_lds(d, env, s);
        emit_obs(d, env, s, o);
    }
}

// action of packet lane l from the 3 A prefetched words: randint(4, size=A) uses word l (mask 3),
// rand(A) words A + 2 l, A + 2 l + 1; first maximum of the (masked) Q row unless the draw < eps
__device__ __forceinline__ int egreedy_lane(const EnvDev& d, const float* q, double eps, size_t p,
                                            const uint32_t* rbuf, int l, int A) {
    const float4 qv = reinterpret_cast<const float4*>(q)[p];
    float v[4] = {qv.x, qv.y, qv.z, qv.w};
    if (d.amask_on) {
        const uint32_t m = reinterpret_cast<const uint32_t*>(d.amask)[p];
        for (int k = 0; k < 4; k++)
            if ((m >> (8 * k)) & 0xffu) v[k] = -__builtin_inff();
    }
    int best = 0;
    for (int k = 1; k < 4; k++)
        if (v[k] > v[best]) best = k;
    const int ra = (int)(rbuf[l] & 3u);
    const uint32_t w0 = rbuf[A + 2 * l], w1 = rbuf[A + 2 * l + 1];
    const double u = ((int32_t)(w0 >> 5) * 67108864.0 + (int32_t)(w1 >> 6)) / 9007199254740992.0;
    return u < eps ? ra : best;
}

struct StepOut {
    float* reward;
    uint8_t* done;
    double* info;
    gm_step_detail det;
    const float* q;    // gm_env_policy_step: Q [n_env, A, 4] -> ε-greedy prologue (nullable)
    double eps;
    int32_t* act_out;  // the actions drawn by the prologue, [n_env, A]
};

// src/env/routing.py:360-520
template <int NC>
__global__ __launch_bounds__(64) void k_env_step(EnvDev d, const int32_t* act, StepOut out, gm_obs_buffers o) {
    const int env = blockIdx.x;
    const int l = lane_id();
    const int N = d.N, A = d.A, E = d.E;
    __shared__ EnvLds<NC> s;
    load_topology_lds(d, env, s);

    // packet a in lane a (registers)
    const bool own = l < A;
    const size_t p = (size_t)env * A + l;
    int now = 0, target = 0, edge = -1, time = 0, ttl = 0, steps = 0, spw = 0, start = 0, a_t = 0;
    double size = 0.0;
    uint64_t vis[2] = {0ull, 0ull};  // visited node set (N <= 128)
    // ε-greedy prologue (gm_policy_egreedy's draws, same stream order: the policy draws before
    // the step's respawns); the stream position stays in registers for the respawn draws below
    int rng_cur = 0, rng_pos = 0, rng_next = 0;
    const bool pol = out.q != nullptr;
    if (pol) {
        MainRng r = open_rng(d, env, s);
        r.prefetch(3 * A);
        if (own) a_t = egreedy_lane(d, out.q, out.eps, p, s.rbuf, l, A);
        r.k = 3 * A;
        close_rng(d, env, r);
        rng_cur = r.cur;
        rng_pos = r.pos;
        rng_next = r.has_next;
        if (own) out.act_out[p] = a_t;
    }
    if (own) {
        now = d.now[p]; target = d.target[p]; edge = d.edge[p]; time = d.time[p];
        ttl = d.ttl_[p]; steps = d.steps[p]; spw = d.spw[p]; start = d.start[p];
        size = d.size[p]; vis[0] = d.visited[p * 2]; vis[1] = d.visited[p * 2 + 1];
        if (!pol) a_t = act[p];
        if (a_t < 0 || a_t > 3) {  // the reference raises IndexError; flag and idle
            atomicExch(d.err, GM_ERR_INVALID_ARG);
            a_t = 0;
        }
    }
    // edge e in lane e % 64, slot e / 64 (E <= 192)
    double ld0 = l < E ? d.load[(size_t)env * E + l] : 0.0;
    double ld1 = l + WAVE < E ? d.load[(size_t)env * E + l + WAVE] : 0.0;
    double ld2 = l + 2 * WAVE < E ? d.load[(size_t)env * E + l + 2 * WAVE] : 0.0;

    steps += 1;  // routing.py:371
    float reward = 0.0f;

    // ---- phase 1 (routing.py:380-412): admission, lower packet id first ----
    int chosen = -1;
    if (own && edge == -1 && a_t != 0) chosen = s.nbr_edge[now * 3 + (a_t - 1)];
    uint64_t admit = 0, block = 0;
    for (int i = 0; i < A; i++) {
        int c = readlane(chosen, i);
        if (c < 0) continue;  // uniform
        double si = readlane_f64(size, i);
        if ((c & (WAVE - 1)) == l) {
            const int slot = c >> 6;
            double ld = slot == 0 ? ld0 : (slot == 1 ? ld1 : ld2);
            if (d.cong && ld + si > 1.0) {
                block |= 1ull << i;
            } else {
                ld = ld + si;
                admit |= 1ull << i;
                if (slot == 0) ld0 = ld;
                else if (slot == 1) ld1 = ld;
                else ld2 = ld;
            }
        }
    }
    admit = wave_or_u64(admit);
    block = wave_or_u64(block);
    bool looped = false;
    if (own) {
        if ((block >> l) & 1ull) reward = reward - 0.2f;
        if ((admit >> l) & 1ull) {
            edge = chosen;
            time = s.elen[chosen];
            now = s.ea[chosen] ^ s.eb[chosen] ^ now;
            if (bit128(vis, now)) looped = true;
            else set128(vis, now);
        }
    }

    // eval-only statistics after admission (routing.py:414-441): sums in edge / packet order
    if (out.det.eval) {
        double tel = 0.0, tps = 0.0;
        int occ = 0;
        for (int e = 0; e < E; e++) {
            double le = e < WAVE ? readlane_f64(ld0, e)
                                 : (e < 2 * WAVE ? readlane_f64(ld1, e - WAVE) : readlane_f64(ld2, e - 2 * WAVE));
            tel = tel + le;
            occ += le > 0.0;
        }
        for (int i = 0; i < A; i++) tps = tps + readlane_f64(size, i);
        const int on_edges = __popcll(ballot(own && edge != -1));
        const int dist = wave_sum_i32(own ? (int)d.apsp[((size_t)env * N + now) * N + target] : 0);
        if (l == 0) {
            double* ev = out.det.eval + (size_t)env * GM_EVAL_FIELDS;
            ev[GM_EVAL_TOTAL_EDGE_LOAD] = tel;
            ev[GM_EVAL_OCCUPIED_EDGES] = (double)occ;
            ev[GM_EVAL_PACKETS_ON_EDGES] = (double)on_edges;
            ev[GM_EVAL_TOTAL_PACKET_SIZE] = tps;
            ev[GM_EVAL_SUM_PACKET_DISTANCES] = (double)dist;
        }
    }

    // ---- phase 2 (routing.py:444-495) ----
    int sub_edge = -1;
    bool drop = false, fin = false, reached = false;
    uint32_t am = 0;
    if (own) {
        am = reinterpret_cast<const uint32_t*>(d.amask)[p];
        ttl -= 1;
        if (edge != -1) {
            time -= 1;
            if (time <= 0) {
                sub_edge = edge;
                edge = -1;
            }
        }
        drop = d.ttl > 0 && ttl <= 0;
        if (d.amask_on) {
            if (edge != -1) {
                am = 0;
            } else {
                am = 1u;
                int cnt = 1;
                for (int k = 0; k < 3; k++) {
                    uint32_t b = (uint32_t)bit128(vis, s.nbr[now * 3 + k]);
                    am |= b << (8 * (k + 1));
                    cnt += (int)b;
                }
                if (cnt == 4) drop = true;
            }
        }
        reached = edge == -1 && now == target;
        fin = reached || drop;
        if (fin) {
            reward = reward + (reached ? 10.0f : -10.0f);
            if (edge != -1) sub_edge = edge;  // reset_packet frees its edge (125-127)
        }
    }
    // loads: per-edge subtraction in packet order
    for (int i = 0; i < A; i++) {
        int c = readlane(sub_edge, i);
        if (c < 0) continue;
        double si = readlane_f64(size, i);
        if (c == l) ld0 = ld0 - si;
        else if (c == l + WAVE) ld1 = ld1 - si;
        else if (c == l + 2 * WAVE) ld2 = ld2 - si;
    }
    // statistics of finished packets (before respawn)
    const int opt = spw > 1 ? spw : 1;
    const int done_steps = fin ? steps : 0;
    uint64_t finm = ballot(own && fin);
    uint64_t succm = ballot(own && fin && reached);
    uint64_t loopm = ballot(own && looped);
    if (out.det.done_steps && own) out.det.done_steps[p] = done_steps;
    if (out.det.done_opt && own) out.det.done_opt[p] = fin ? opt : 0;
    if (out.det.success && own) out.det.success[p] = (uint8_t)(fin && reached);
    if (out.info) {
        int sd = wave_sum_i32(fin ? steps : 0);
        int sda = wave_sum_i32(fin && reached ? steps : 0);
        double spr_sum = 0.0;
        for (int i = 0; i < A; i++) {  // in packet order, like the reference's list
            if (!((succm >> i) & 1ull)) continue;
            int st = readlane(steps, i), op = readlane(opt, i);
            spr_sum += (double)st / (double)op;
        }
        if (l == 0) {
            double* inf = out.info + (size_t)env * GM_INFO_FIELDS;
            inf[GM_INFO_LOOPED] = (double)__popcll(loopm);
            inf[GM_INFO_THROUGHPUT] = (double)__popcll(succm);
            inf[GM_INFO_DROPPED] = (double)__popcll(finm & ~succm);
            inf[GM_INFO_BLOCKED] = (double)__popcll(block);
            inf[GM_INFO_N_DELAYS] = (double)__popcll(finm);
            inf[GM_INFO_SUM_DELAYS] = (double)sd;
            inf[GM_INFO_N_ARRIVED] = (double)__popcll(succm);
            inf[GM_INFO_SUM_DELAYS_ARRIVED] = (double)sda;
            inf[GM_INFO_SUM_SPR] = spr_sum;
        }
    }
    if (own) {
        out.reward[p] = reward;
        out.done[p] = (uint8_t)fin;
    }
    // respawn finished packets in id order (reset_packet draws, routing.py:130-134)
    if (finm) {
        MainRng r = open_rng(d, env, s);
        if (pol) {  // the prologue's position (its lane-0 stores are not read back)
            r.cur = rng_cur;
            r.pos = rng_pos;
            r.has_next = rng_next;
        }
        r.prefetch(6 * __popcll(finm) + 8);
        uint64_t m = finm;
        while (m) {
            int i = __builtin_ctzll(m);
            m &= m - 1;
            int st = (int)r.randint(N);
            int tg = (int)r.randint(N);
            double sz = r.random();
            if (l == i) {
                now = st;
                target = tg;
                size = sz;
                start = st;
            }
        }
        close_rng(d, env, r);
        if (own && fin) {
            time = 0;
            edge = -1;
            ttl = d.ttl;
            steps = 0;
            spw = d.apsp[((size_t)env * N + now) * N + target];
            vis[0] = 0ull;
            vis[1] = 0ull;
            set128(vis, now);
            am = d.amask_on ? (uint32_t)(now != target) : 0u;
        }
    }
    // write back
    if (own) {
        d.now[p] = now; d.target[p] = target; d.edge[p] = edge; d.time[p] = time;
        d.ttl_[p] = ttl; d.steps[p] = steps; d.spw[p] = spw; d.start[p] = start;
        d.size[p] = size; d.visited[p * 2] = vis[0]; d.visited[p * 2 + 1] = vis[1];
        reinterpret_cast<uint32_t*>(d.amask)[p] = am;
        s.now[l] = now; s.target[l] = target; s.edge[l] = edge; s.time[l] = time; s.size[l] = size;
    }
    if (l < E) { d.load[(size_t)env * E + l] = ld0; s.load[l] = ld0; }
    if (l + WAVE < E) { d.load[(size_t)env * E + l + WAVE] = ld1; s.load[l + WAVE] = ld1; }
    if (l + 2 * WAVE < E) { d.load[(size_t)env * E + l + 2 * WAVE] = ld2; s.load[l + 2 * WAVE] = ld2; }
    __syncthreads();
    if (o.obs || o.obs_gemm || o.node_obs || o.agent_node || o.agent_adj) emit_obs(d, env, s, o);
}

template <int NC>
__global__ __launch_bounds__(64) void k_env_observe(EnvDev d, gm_obs_buffers o) {
    const int env = blockIdx.x;
    __shared__ EnvLds<NC> s;
    load_topology_lds(d, env, s);
    load_packets_lds(d, env, s);
    emit_obs(d, env, s, o);
}

// obs rows from the GEMM-ready copy (gm_obs_from_gemm): one wave per row, lane l writes 16-B
// chunk l of the 6N+10 columns (the last one a float2: 6N+10 = 4q+2 for even N). Copy column c
// comes from obs column c (c < N-1), c+1 (c < 2N-1), c+2 (else), so obs column j reads copy
// column j (j < N-1), j-1 (N <= j < 2N), j-2 (j > 2N); column N-1 is the target one-hot's sum
// minus the other position one-hots, column 2N the next-hop one-hot's sum (0 / 1 sums: exact)
__global__ __launch_bounds__(256) void k_obs_from_gemm(const float* __restrict__ g, long long ldg, long long rows, int N,
                                                       float* __restrict__ obs, long long ldo) {
    const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int l = threadIdx.x & 63;
    const float* gr = g + r * ldg;
    float* orow = obs + r * ldo;
    const int D1 = 6 * N + 10, Q = (D1 + 3) / 4;
    float pos = 0.f, tgt = 0.f, hop = 0.f;  // wave sums of the one-hot blocks
    for (int c = l; c < N - 1; c += 64) pos += gr[c];
    for (int c = N - 1 + l; c < 2 * N - 1; c += 64) tgt += gr[c];
    for (int c = 2 * N - 1 + l; c < 3 * N - 1; c += 64) hop += gr[c];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        pos += __shfl_xor(pos, o);
        tgt += __shfl_xor(tgt, o);
        hop += __shfl_xor(hop, o);
    }
    for (int q = l; q < Q; q += 64) {
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int c = 4 * q + j;
            v[j] = c < N - 1 ? gr[c] : c == N - 1 ? tgt - pos : c < 2 * N ? gr[c - 1] : c == 2 * N ? hop
                 : c < D1 ? gr[c - 2] : 0.f;
        }
        if (4 * q + 4 <= D1)
            *reinterpret_cast<float4*>(orow + 4 * q) = make_float4(v[0], v[1], v[2], v[3]);
        else
            *reinterpret_cast<float2*>(orow + 4 * q) = make_float2(v[0], v[1]);
    }
}

// EpsilonGreedy.__call__ (src/policy.py:20-64): randint(4, size=A) then rand(A)
// from the env's stream every call; argmax (first maximum) unless the draw < eps.
__global__ __launch_bounds__(64) void k_policy_egreedy(EnvDev d, const float* q, double eps, int32_t* actions) {
    const int env = blockIdx.x;
    const int l = lane_id();
    const int A = d.A;
    __shared__ uint32_t rbuf[RNG_BUF];
    __shared__ uint32_t rtmp[MT_N];
    MainRng r;
    r.g = d.mt + (size_t)env * 2 * MT_N;
    r.buf = rbuf;
    r.tmp = rtmp;
    r.cur = d.mt_cur[env];
    r.pos = d.mt_pos[env];
    r.has_next = d.mt_has_next[env];
    r.n = 0;
    r.k = 0;
    r.prefetch(3 * A);
    if (l < A) {
        size_t p = (size_t)env * A + l;
        actions[p] = egreedy_lane(d, q, eps, p, rbuf, l, A);
    }
    r.k = 3 * A;
    r.commit();
    if (l == 0) {
        d.mt_cur[env] = r.cur;
        d.mt_pos[env] = r.pos;
        d.mt_has_next[env] = r.has_next;
    }
}

// ShortestPath heuristic (src/policy.py:90-139): each packet takes the first hop of
// networkx's weighted shortest path (nx.shortest_path(G, weight="weight"),
// src/env/network.py:279) towards its target. Lane s runs networkx's Dijkstra from
// source s with its exact tie-breaking: the heap pops the smallest (distance, push
// counter); a node's path is replaced only on a strictly shorter distance; neighbours
// are relaxed in G's adjacency order = edge creation order (network.py:179-186).
// Only the latest push of a node can be live, so the heap is the per-node
// (seen, counter) pair. first[s][t] = first hop on the s -> t path.
// LDS: first 16 KB + seen/cnt 32 KB + the topology image.
template <int NC>
struct FirstHopLds {
    EnvLds<NC> s;
    uint8_t first[NC * NC];
    int16_t seen[NC * WAVE];
    int16_t cnt[NC * WAVE];
};

template <class FS>
__device__ void first_hops_lds(const EnvDev& d, int env, FS& F) {
    const int l = lane_id();
    const int N = d.N;
    auto& s = F.s;
    uint8_t* first = F.first;
    int16_t* seen = F.seen;
    int16_t* cnt = F.cnt;
    load_topology_lds(d, env, s);
    constexpr int16_t INF = 0x7fff;
    for (int src = l; src < N; src += WAVE) {  // lane l runs sources l and l + 64
        for (int u = 0; u < N; u++) seen[u * WAVE + l] = INF;
        seen[src * WAVE + l] = 0;
        cnt[src * WAVE + l] = 0;
        first[src * N + src] = (uint8_t)src;
        int c = 1;
        uint64_t done[2] = {0ull, 0ull};
        for (int it = 0; it < N; it++) {
            int v = -1, bd = INF, bc = 0;
            for (int u = 0; u < N; u++) {
                if (bit128(done, u)) continue;
                const int du = seen[u * WAVE + l];
                if (du == INF) continue;
                const int cu = cnt[u * WAVE + l];
                if (v < 0 || du < bd || (du == bd && cu < bc)) {
                    v = u;
                    bd = du;
                    bc = cu;
                }
            }
            if (v < 0) break;
            set128(done, v);
            int e3[3] = {s.nbr_edge[v * 3], s.nbr_edge[v * 3 + 1], s.nbr_edge[v * 3 + 2]};
            for (int i = 1; i < 3; i++)  // incident edges in creation (edge id) order
                for (int j = i; j > 0 && e3[j] < e3[j - 1]; j--) {
                    int t = e3[j];
                    e3[j] = e3[j - 1];
                    e3[j - 1] = t;
                }
            for (int k = 0; k < 3; k++) {
                const int e = e3[k];
                const int u = s.ea[e] ^ s.eb[e] ^ v;
                if (bit128(done, u)) continue;
                const int vu = bd + (int)s.elen[e];
                const int su = seen[u * WAVE + l];
                if (su == INF || vu < su) {
                    seen[u * WAVE + l] = (int16_t)vu;
                    cnt[u * WAVE + l] = (int16_t)c++;
                    first[src * N + u] = v == src ? (uint8_t)u : first[src * N + v];
                }
            }
        }
    }
    __syncthreads();
}

template <int NC>
__global__ __launch_bounds__(64) void k_policy_shortest_path(EnvDev d, int32_t* actions) {
    const int env = blockIdx.x;
    const int l = lane_id();
    const int N = d.N, A = d.A;
    __shared__ FirstHopLds<NC> F;
    first_hops_lds(d, env, F);
    auto& s = F.s;
    const uint8_t* first = F.first;
    if (l < A) {
        const size_t p = (size_t)env * A + l;
        const int now = d.now[p], target = d.target[p];
        int a = 0;
        if (now != target) {
            const int nx = first[now * N + target];
            for (int k = 0; k < 3; k++)
                if (s.nbr[now * 3 + k] == nx) {
                    a = k + 1;
                    break;
                }
        }
        actions[p] = a;
    }
}

template <int NC>
__global__ __launch_bounds__(64) void k_env_first_hops(EnvDev d, int32_t* out) {
    const int env = blockIdx.x;
    __shared__ FirstHopLds<NC> F;
    first_hops_lds(d, env, F);
    const int N = d.N;
    for (int i = lane_id(); i < N * N; i += WAVE) out[(size_t)env * N * N + i] = F.first[i];
}

__global__ void k_rng_seed(EnvDev d, const uint32_t* seeds) {
    int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= d.n_env) return;
    uint32_t* k = d.mt + (size_t)env * 2 * MT_N;
    uint32_t v = seeds[env];
    k[0] = v;
    for (int i = 1; i < MT_N; i++) {
        v = 1812433253u * (v ^ (v >> 30)) + (uint32_t)i;
        k[i] = v;
    }
    d.mt_cur[env] = 0;
    d.mt_pos[env] = MT_N;
    d.mt_has_next[env] = 0;
    d.seq_index[env] = 0;
    d.topo_ready[env] = 0;
}

__global__ void k_topology_out(EnvDev d, int32_t* nbr, int8_t* node_adj, float* node_aux, int64_t* seeds) {
    const int env = blockIdx.x;
    const int l = threadIdx.x;
    const int N = d.N;
    if (nbr)
        for (int i = l; i < N * 3; i += blockDim.x) nbr[(size_t)env * N * 3 + i] = d.nbr[(size_t)env * N * 3 + i];
    if (node_adj) {
        for (int idx = l; idx < N * N; idx += blockDim.x) {
            int i = idx / N, j = idx % N;
            const int32_t* nb = d.nbr + ((size_t)env * N + i) * 3;
            node_adj[(size_t)env * N * N + idx] = (int8_t)(i == j || nb[0] == j || nb[1] == j || nb[2] == j);
        }
    }
    if (node_aux)
        for (int idx = l; idx < N * N; idx += blockDim.x)
            node_aux[(size_t)env * N * N + idx] = (float)d.apsp[(size_t)env * N * N + idx];
    if (seeds && l == 0) seeds[env] = d.topo_seed[env];
}

__global__ void k_final_info(EnvDev d, double* out) {
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= d.n_env) return;
    double s = 0.0, c = 0.0;
    for (int a = 0; a < d.A; a++) {
        int st = d.steps[(size_t)env * d.A + a];
        if (st != 0) {
            s += st;
            c += 1.0;
        }
    }
    out[env * 2] = s;
    out[env * 2 + 1] = c;
}

// src/env/network.py:100-120 build_seed_list: main stream seeded with the init seed;
// each candidate seed is a main-stream draw (exclusions re-drawn), its topology chain
// (reseeding on invalid graphs) gives the final seed; unique seeds in order.
constexpr int MAX_SEED_LIST = 4096;

template <int NC>
struct SeedListLds {
    EnvLds<NC> env;
    TopoLds<NC> topo;
};

template <int NC>
__global__ __launch_bounds__(64) void k_build_seed_list(EnvDev d, int count, int64_t* out) {
    __shared__ SeedListLds<NC> S;
    __shared__ int64_t found[MAX_SEED_LIST];
    MainRng r = open_rng(d, 0, S.env);
    int have = 0;
    // duplicates are rare (2^31 seeds); a bounded candidate budget keeps a broken
    // stream from spinning forever
    for (int cands = 0; have < count; cands++) {
        if (cands > 64 * count + 1024) {
            if (lane_id() == 0) atomicExch(d.err, GM_ERR_TOPOLOGY);
            break;
        }
        int64_t cand = draw_topology_seed(d, r);
        r.commit();
        LocalRng tr;
        tr.key = S.topo.tkey;
        tr.seed((uint32_t)cand);
        int64_t seed = cand;
        int reps = 0;
        for (;;) {
            bool ok = topology_attempt(d, S.topo, tr);
            reps++;
            if (ok || reps > 100000) break;
            seed = draw_topology_seed(d, tr);
            tr.seed((uint32_t)seed);
        }
        bool dup = false;
        for (int i = 0; i < have; i++) dup |= found[i] == seed;
        __syncthreads();
        if (!dup) {
            if (lane_id() == 0) found[have] = seed;
            have++;
        }
        __syncthreads();
    }
    for (int i = lane_id(); i < have; i += WAVE) out[i] = found[i];
    close_rng(d, 0, r);
}

inline int ncap(int n) { return n <= 64 ? 64 : 128; }

bool has_obs(const gm_obs_buffers* o) {
    return o && (o->obs || o->obs_gemm || o->node_obs || o->agent_node || o->agent_adj);
}

int check_launch() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return GM_OK;
}

template <class T>
int dalloc(gm_env* env, T** p, size_t n) {
    void* q = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&q, n * sizeof(T));
    if (e != hipSuccess) return gm_fail(GM_ERR_OOM, std::string("hipMalloc: ") + hipGetErrorString(e));
    env->allocs.push_back(q);
    *p = (T*)q;
    return GM_OK;
}

}  // namespace

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
extern "C" int gm_env_destroy(gm_env* env) {
    if (!env) return GM_OK;
    (void)hipSetDevice(env->device);
    for (void* p : env->allocs) (void)hipFree(p);
    delete env;
    return GM_OK;
}

extern "C" int gm_env_create(const gm_env_config* cfg, const uint32_t* env_seeds, gm_env** out) {
    if (!cfg || !env_seeds || !out) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    const int N = cfg->n_nodes, A = cfg->n_data;
    if (cfg->n_env <= 0) return gm_fail(GM_ERR_INVALID_ARG, "n_env must be > 0");
    if (N < 4 || N > MAX_NODES || (N % 2) != 0)
        return gm_fail(GM_ERR_INVALID_ARG, "n_nodes must be even and in [4, 128] (3-regular topology generator)");
    if (A < 1 || A > MAX_AGENTS) return gm_fail(GM_ERR_INVALID_ARG, "n_data must be in [1, 64]");
    if (cfg->env_var < 1 || cfg->env_var > 3) return gm_fail(GM_ERR_INVALID_ARG, "env_var must be 1, 2 or 3");
    if (cfg->env_var == 2 && (cfg->k < 0 || cfg->k > MAX_KNBR))
        return gm_fail(GM_ERR_INVALID_ARG, "k (variant-2 neighbours) must be in [0, 8]");
    if ((cfg->topo_mode == GM_TOPO_LIST || cfg->topo_mode == GM_TOPO_SEQUENTIAL) &&
        (cfg->n_seed_list <= 0 || !cfg->seed_list))
        return gm_fail(GM_ERR_INVALID_ARG, "seed list required for LIST/SEQUENTIAL topology mode");
    if (cfg->topo_mode < 0 || cfg->topo_mode > 3) return gm_fail(GM_ERR_INVALID_ARG, "bad topo_mode");
    GM_HIP(hipSetDevice(cfg->device));
    gm_env* env = new gm_env();
    env->cfg = *cfg;
    env->device = cfg->device;
    if (cfg->seed_list) env->list.assign(cfg->seed_list, cfg->seed_list + cfg->n_seed_list);
    if (cfg->excluded) {
        env->excl.assign(cfg->excluded, cfg->excluded + cfg->n_excluded);
        std::sort(env->excl.begin(), env->excl.end());
    }
    env->cfg.seed_list = nullptr;
    env->cfg.excluded = nullptr;
    EnvDev& d = env->d;
    memset(&d, 0, sizeof(d));
    const size_t B = (size_t)cfg->n_env;
    d.n_env = cfg->n_env;
    d.N = N;
    d.A = A;
    d.E = 3 * N / 2;
    d.env_var = cfg->env_var;
    d.k = cfg->env_var == 2 ? cfg->k : 0;
    d.cong = cfg->congestion != 0;
    d.amask_on = cfg->action_mask != 0;
    d.ttl = cfg->ttl;
    d.topo_mode = cfg->topo_mode;
    d.fixed_seed = cfg->topo_seed;
    d.n_list = (int)env->list.size();
    d.n_excl = (int)env->excl.size();
    d.seq_stride = 1;
    int rc = GM_OK;
#define ALLOC(ptr, n) \
    if ((rc = dalloc(env, &(ptr), (n))) != GM_OK) { gm_env_destroy(env); return rc; }
    int64_t *list_d = nullptr, *excl_d = nullptr;
    ALLOC(list_d, env->list.size());
    ALLOC(excl_d, env->excl.size());
    d.list = list_d;
    d.excl = excl_d;
    ALLOC(d.nbr, B * N * 3);
    ALLOC(d.nbr_edge, B * N * 3);
    ALLOC(d.edge_a, B * d.E);
    ALLOC(d.edge_b, B * d.E);
    ALLOC(d.edge_len, B * d.E);
    ALLOC(d.apsp, B * N * N);
    ALLOC(d.topo_seed, B);
    ALLOC(d.topo_reps, B);
    ALLOC(d.topo_ready, B);
    ALLOC(d.seq_index, B);
    ALLOC(d.now, B * A);
    ALLOC(d.target, B * A);
    ALLOC(d.edge, B * A);
    ALLOC(d.time, B * A);
    ALLOC(d.ttl_, B * A);
    ALLOC(d.start, B * A);
    ALLOC(d.spw, B * A);
    ALLOC(d.steps, B * A);
    ALLOC(d.size, B * A);
    ALLOC(d.visited, B * A * 2);
    ALLOC(d.amask, B * A * 4);
    ALLOC(d.load, B * d.E);
    ALLOC(d.mt, B * 2 * MT_N);
    ALLOC(d.mt_cur, B);
    ALLOC(d.mt_pos, B);
    ALLOC(d.mt_has_next, B);
    ALLOC(d.err, 1);
    uint32_t* seeds_d = nullptr;
    ALLOC(seeds_d, B);
#undef ALLOC
    GM_HIP(hipMemcpy(seeds_d, env_seeds, B * sizeof(uint32_t), hipMemcpyHostToDevice));
    if (!env->list.empty())
        GM_HIP(hipMemcpy(list_d, env->list.data(), env->list.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    if (!env->excl.empty())
        GM_HIP(hipMemcpy(excl_d, env->excl.data(), env->excl.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    GM_HIP(hipMemset(d.err, 0, sizeof(int32_t)));
    GM_HIP(hipMemset(d.edge, 0xff, B * A * sizeof(int32_t)));
    GM_HIP(hipMemset(d.load, 0, B * d.E * sizeof(double)));
    GM_HIP(hipMemset(d.steps, 0, B * A * sizeof(int32_t)));
    GM_HIP(hipMemset(d.amask, 0, B * A * 4));
    hipLaunchKernelGGL(k_rng_seed, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, 0, d, seeds_d);
    if ((rc = check_launch()) != GM_OK) { gm_env_destroy(env); return rc; }
    GM_HIP(hipDeviceSynchronize());
    *out = env;
    return GM_OK;
}

extern "C" int gm_env_dims(const gm_env* env, int32_t* n_env, int32_t* n_nodes, int32_t* n_data, int32_t* obs_dim,
                           int32_t* node_obs_dim) {
    if (!env) return gm_fail(GM_ERR_INVALID_ARG, "null env");
    if (n_env) *n_env = env->d.n_env;
    if (n_nodes) *n_nodes = env->d.N;
    if (n_data) *n_data = env->d.A;
    if (obs_dim) *obs_dim = obs_dim_of(env->d.N, env->d.env_var, env->d.k);
    if (node_obs_dim) *node_obs_dim = 4 * env->d.N + 8;
    return GM_OK;
}

static int check_obs(const gm_env* env, const gm_obs_buffers* o) {
    if (o && o->obs && o->obs_row_stride < obs_dim_of(env->d.N, env->d.env_var, env->d.k))
        return gm_fail(GM_ERR_INVALID_ARG, "obs_row_stride smaller than the observation size");
    if (o && o->obs_gemm &&
        (env->d.env_var != 1 || (env->d.N & 1) || o->obs_gemm_stride < 6 * env->d.N + 8 ||
         (o->obs_gemm_stride % 4) || (reinterpret_cast<uintptr_t>(o->obs_gemm) & 15)))
        // the copy is written as (6N+8)/4 whole float4 chunks per row: N must be even
        return gm_fail(GM_ERR_INVALID_ARG, "obs_gemm: env_var 1, even N, stride >= 6N+8 and 16-byte rows");
    return GM_OK;
}

extern "C" int gm_env_reset(gm_env* env, const uint8_t* reset_mask, const gm_obs_buffers* obs, void* stream) {
    if (!env) return gm_fail(GM_ERR_INVALID_ARG, "null env");
    int rc = check_obs(env, obs);
    if (rc) return rc;
    gm_obs_buffers o = obs ? *obs : gm_obs_buffers{};
    // N <= 32: the 32-node LDS image (14 KB instead of 24 KB per env) doubles the envs per CU
    if (env->d.N <= 32) hipLaunchKernelGGL(k_env_reset<32>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, reset_mask, o);
    else if (ncap(env->d.N) == 64) hipLaunchKernelGGL(k_env_reset<64>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, reset_mask, o);
    else hipLaunchKernelGGL(k_env_reset<128>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, reset_mask, o);
    return check_launch();
}

static int launch_step(gm_env* env, const int32_t* actions, const float* q, double epsilon, int32_t* act_out,
                       float* reward, uint8_t* done, double* info, const gm_step_detail* detail,
                       const gm_obs_buffers* obs, void* stream) {
    int rc = check_obs(env, obs);
    if (rc) return rc;
    StepOut so;
    so.reward = reward;
    so.done = done;
    so.info = info;
    so.det = detail ? *detail : gm_step_detail{};
    so.q = q;
    so.eps = epsilon;
    so.act_out = act_out;
    gm_obs_buffers o = obs ? *obs : gm_obs_buffers{};
    if (ncap(env->d.N) == 64) hipLaunchKernelGGL(k_env_step<64>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, actions, so, o);
    else hipLaunchKernelGGL(k_env_step<128>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, actions, so, o);
    return check_launch();
}

extern "C" int gm_env_step(gm_env* env, const int32_t* actions, float* reward, uint8_t* done, double* info,
                           const gm_step_detail* detail, const gm_obs_buffers* obs, void* stream) {
    if (!env || !actions || !reward || !done) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    return launch_step(env, actions, nullptr, 0.0, nullptr, reward, done, info, detail, obs, stream);
}

extern "C" int gm_env_policy_step(gm_env* env, const float* q, double epsilon, int32_t* actions, float* reward,
                                  uint8_t* done, double* info, const gm_step_detail* detail, const gm_obs_buffers* obs,
                                  void* stream) {
    if (!env || !q || !actions || !reward || !done) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    if ((reinterpret_cast<uintptr_t>(q) & 15) != 0) return gm_fail(GM_ERR_INVALID_ARG, "q must be 16-byte aligned");
    return launch_step(env, nullptr, q, epsilon, actions, reward, done, info, detail, obs, stream);
}

__global__ void k_topology_rewind(EnvDev d, int interleave) {
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= d.n_env) return;
    d.seq_index[env] = interleave ? env % d.n_list : 0;
    d.topo_ready[env] = 0;
}

extern "C" int gm_policy_shortest_path(gm_env* env, int32_t* actions, void* stream) {
    if (!env || !actions) return gm_fail(GM_ERR_INVALID_ARG, "gm_policy_shortest_path: null argument");
    if (ncap(env->d.N) == 64) hipLaunchKernelGGL(k_policy_shortest_path<64>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, actions);
    else hipLaunchKernelGGL(k_policy_shortest_path<128>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, actions);
    return check_launch();
}

extern "C" int gm_env_first_hops(gm_env* env, int32_t* out, void* stream) {
    if (!env || !out) return gm_fail(GM_ERR_INVALID_ARG, "gm_env_first_hops: null argument");
    if (ncap(env->d.N) == 64) hipLaunchKernelGGL(k_env_first_hops<64>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, out);
    else hipLaunchKernelGGL(k_env_first_hops<128>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, out);
    return check_launch();
}

extern "C" int gm_env_set_topology(gm_env* env, int32_t topo_mode, int64_t topo_seed, const int64_t* seed_list,
                                   int32_t n_seed_list, int32_t interleave) {
    if (!env || topo_mode < 0 || topo_mode > 3) return gm_fail(GM_ERR_INVALID_ARG, "gm_env_set_topology: bad mode");
    if ((topo_mode == GM_TOPO_LIST || topo_mode == GM_TOPO_SEQUENTIAL) && (n_seed_list <= 0 || !seed_list))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_env_set_topology: seed list required for LIST/SEQUENTIAL");
    GM_HIP(hipSetDevice(env->device));
    GM_HIP(hipDeviceSynchronize());  // no reset in flight reads the old list
    EnvDev& d = env->d;
    if (n_seed_list > 0 && seed_list) {
        env->list.assign(seed_list, seed_list + n_seed_list);
        int64_t* list_d = nullptr;
        int rc = dalloc(env, &list_d, env->list.size());
        if (rc != GM_OK) return rc;
        GM_HIP(hipMemcpy(list_d, env->list.data(), env->list.size() * sizeof(int64_t), hipMemcpyHostToDevice));
        d.list = list_d;
        d.n_list = (int)env->list.size();
    }
    d.topo_mode = topo_mode;
    d.fixed_seed = topo_seed;
    env->cfg.topo_mode = topo_mode;
    env->cfg.topo_seed = topo_seed;
    d.seq_stride = interleave ? d.n_env : 1;
    hipLaunchKernelGGL(k_topology_rewind, dim3((unsigned)((d.n_env + 63) / 64)), dim3(64), 0, 0, d,
                       (int)(interleave && d.n_list > 0));
    int rc = check_launch();
    if (rc != GM_OK) return rc;
    GM_HIP(hipDeviceSynchronize());
    return GM_OK;
}

extern "C" int gm_env_observe(gm_env* env, const gm_obs_buffers* obs, void* stream) {
    if (!env) return gm_fail(GM_ERR_INVALID_ARG, "null env");
    if (!has_obs(obs)) return GM_OK;
    int rc = check_obs(env, obs);
    if (rc) return rc;
    if (ncap(env->d.N) == 64) hipLaunchKernelGGL(k_env_observe<64>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, *obs);
    else hipLaunchKernelGGL(k_env_observe<128>, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, *obs);
    return check_launch();
}

extern "C" int gm_obs_from_gemm(const float* obs_gemm, int64_t ld_gemm, int64_t rows, int32_t n_nodes, float* obs,
                                int64_t ld_obs, void* stream) {
    if (!obs_gemm || !obs || rows < 0 || n_nodes < 2 || (n_nodes & 1) || ld_gemm < 6 * n_nodes + 8 || (ld_gemm % 4) ||
        ld_obs < 6 * n_nodes + 10 || (ld_obs % 4) || (reinterpret_cast<uintptr_t>(obs) & 15))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_obs_from_gemm: even N, ld_gemm >= 6N+8, ld_obs >= 6N+10, 16-byte rows");
    if (rows == 0) return GM_OK;
    hipLaunchKernelGGL(k_obs_from_gemm, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, obs_gemm,
                       (long long)ld_gemm, (long long)rows, (int)n_nodes, obs, (long long)ld_obs);
    return check_launch();
}

extern "C" int gm_env_topology(gm_env* env, int32_t* nbr, int8_t* node_adj, float* node_aux, int64_t* topo_seed,
                               void* stream) {
    if (!env) return gm_fail(GM_ERR_INVALID_ARG, "null env");
    hipLaunchKernelGGL(k_topology_out, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, nbr, node_adj,
                       node_aux, topo_seed);
    return check_launch();
}

extern "C" int gm_env_final_info(gm_env* env, double* out, void* stream) {
    if (!env || !out) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    hipLaunchKernelGGL(k_final_info, dim3((env->d.n_env + 63) / 64), dim3(64), 0, (hipStream_t)stream, env->d, out);
    return check_launch();
}

extern "C" int gm_policy_egreedy(gm_env* env, const float* q, double epsilon, int32_t* actions, void* stream) {
    if (!env || !q || !actions) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    if ((reinterpret_cast<uintptr_t>(q) & 15) != 0) return gm_fail(GM_ERR_INVALID_ARG, "q must be 16-byte aligned");
    hipLaunchKernelGGL(k_policy_egreedy, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, q, epsilon,
                       actions);
    return check_launch();
}

extern "C" int gm_build_seed_list(int32_t n_nodes, int64_t init_seed, int32_t count, const int64_t* excluded,
                                  int32_t n_excluded, int32_t device, int64_t* out) {
    if (!out || count <= 0 || count > 4096)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_build_seed_list: count must be in [1, 4096]");
    gm_env_config c;
    memset(&c, 0, sizeof(c));
    c.n_env = 1;
    c.n_nodes = n_nodes;
    c.n_data = 1;
    c.env_var = 1;
    c.topo_mode = GM_TOPO_RANDOM;
    c.excluded = excluded;
    c.n_excluded = n_excluded;
    c.device = device;
    uint32_t s0 = (uint32_t)init_seed;
    gm_env* env = nullptr;
    int rc = gm_env_create(&c, &s0, &env);
    if (rc) return rc;
    int64_t* dout = nullptr;
    if ((rc = dalloc(env, &dout, (size_t)count)) != GM_OK) {
        gm_env_destroy(env);
        return rc;
    }
    if (ncap(env->d.N) == 64) hipLaunchKernelGGL(k_build_seed_list<64>, dim3(1), dim3(64), 0, 0, env->d, count, dout);
    else hipLaunchKernelGGL(k_build_seed_list<128>, dim3(1), dim3(64), 0, 0, env->d, count, dout);
    rc = check_launch();
    if (rc == GM_OK) {
        hipError_t e = hipMemcpy(out, dout, (size_t)count * sizeof(int64_t), hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = gm_fail(GM_ERR_HIP, std::string("gm_build_seed_list: ") + hipGetErrorString(e));
        int32_t err = 0;
        if (rc == GM_OK && hipMemcpy(&err, env->d.err, sizeof(err), hipMemcpyDeviceToHost) == hipSuccess && err)
            rc = gm_fail(GM_ERR_TOPOLOGY, "gm_build_seed_list: candidate budget exhausted");
    }
    gm_env_destroy(env);
    return rc;
}

template <class T>
static int d2h(T* host, const T* dev, size_t n) {
    if (!host) return GM_OK;
    GM_HIP(hipMemcpy(host, dev, n * sizeof(T), hipMemcpyDeviceToHost));
    return GM_OK;
}

extern "C" int gm_env_get_state(gm_env* env, gm_env_state* st) {
    if (!env || !st) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    GM_HIP(hipSetDevice(env->device));
    GM_HIP(hipDeviceSynchronize());
    int32_t err = 0;
    GM_HIP(hipMemcpy(&err, env->d.err, sizeof(err), hipMemcpyDeviceToHost));
    if (err) return gm_fail(err, "device reported an invalid topology seed / generator failure");
    const EnvDev& d = env->d;
    const size_t B = d.n_env, A = d.A, N = d.N, E = d.E;
    int rc = 0;
    if ((rc = d2h(st->now, d.now, B * A)) || (rc = d2h(st->target, d.target, B * A)) ||
        (rc = d2h(st->edge, d.edge, B * A)) || (rc = d2h(st->time, d.time, B * A)) ||
        (rc = d2h(st->ttl, d.ttl_, B * A)) || (rc = d2h(st->start, d.start, B * A)) ||
        (rc = d2h(st->spw, d.spw, B * A)) || (rc = d2h(st->agent_steps, d.steps, B * A)) ||
        (rc = d2h(st->size, d.size, B * A)) || (rc = d2h(st->visited, d.visited, B * A * 2)) ||
        (rc = d2h(st->amask, d.amask, B * A * 4)) || (rc = d2h(st->loads, d.load, B * E)) ||
        (rc = d2h(st->topo_seed, d.topo_seed, B)) || (rc = d2h(st->topo_reps, d.topo_reps, B)) ||
        (rc = d2h(st->edge_a, d.edge_a, B * E)) || (rc = d2h(st->edge_b, d.edge_b, B * E)) ||
        (rc = d2h(st->edge_len, d.edge_len, B * E)) || (rc = d2h(st->nbr_edge, d.nbr_edge, B * N * 3)) ||
        (rc = d2h(st->seq_index, d.seq_index, B)))
        return rc;
    if (st->apsp) {
        std::vector<int16_t> tmp(B * N * N);
        GM_HIP(hipMemcpy(tmp.data(), d.apsp, tmp.size() * sizeof(int16_t), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < tmp.size(); i++) st->apsp[i] = tmp[i];
    }
    if (st->rng_key || st->rng_pos) {
        // numpy's view of the stream: the block being consumed and the position in it
        std::vector<uint32_t> mt(B * 2 * MT_N);
        std::vector<int32_t> cur(B), pos(B);
        GM_HIP(hipMemcpy(mt.data(), d.mt, mt.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
        GM_HIP(hipMemcpy(cur.data(), d.mt_cur, B * sizeof(int32_t), hipMemcpyDeviceToHost));
        GM_HIP(hipMemcpy(pos.data(), d.mt_pos, B * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (size_t b = 0; b < B; b++) {
            if (st->rng_key) memcpy(st->rng_key + b * MT_N, mt.data() + (b * 2 + cur[b]) * MT_N, MT_N * 4);
            if (st->rng_pos) st->rng_pos[b] = pos[b];
        }
    }
    return GM_OK;
}

template <typename T>
static int h2d(T* dev, const T* host, size_t n) {
    if (!host) return GM_OK;
    GM_HIP(hipMemcpy(dev, host, n * sizeof(T), hipMemcpyHostToDevice));
    return GM_OK;
}

// Inverse of gm_env_get_state (parity dumps / restores): every non-NULL field is written back;
// the neighbour table is rebuilt from the edge arrays, the numpy stream is restored as block 0
// at rng_pos with no pre-twisted next block (pos 624 = twist before the next draw, as numpy).
// Observation buffers are not touched: call gm_env_observe afterwards.
extern "C" int gm_env_set_state(gm_env* env, const gm_env_state* st) {
    if (!env || !st) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    GM_HIP(hipSetDevice(env->device));
    GM_HIP(hipDeviceSynchronize());
    EnvDev& d = env->d;
    const size_t B = d.n_env, A = d.A, N = d.N, E = d.E;
    if (st->rng_pos)
        for (size_t b = 0; b < B; b++)
            if (st->rng_pos[b] < 0 || st->rng_pos[b] > (int32_t)MT_N)
                return gm_fail(GM_ERR_INVALID_ARG, "gm_env_set_state: rng_pos outside [0, 624]");
    if (st->seq_index)
        for (size_t b = 0; b < B; b++)
            if (st->seq_index[b] < 0 || (d.n_list > 0 && st->seq_index[b] >= d.n_list))
                return gm_fail(GM_ERR_INVALID_ARG, "gm_env_set_state: seq_index outside the topology-seed list");
    if (st->nbr_edge && (!st->edge_a || !st->edge_b))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_env_set_state: nbr_edge needs edge_a and edge_b");
    if (st->nbr_edge)
        for (size_t i = 0; i < B * N * 3; i++)
            if (st->nbr_edge[i] < -1 || st->nbr_edge[i] >= (int32_t)E)
                return gm_fail(GM_ERR_INVALID_ARG, "gm_env_set_state: nbr_edge entry outside [-1, E)");
    int rc = 0;
    if ((rc = h2d(d.now, st->now, B * A)) || (rc = h2d(d.target, st->target, B * A)) ||
        (rc = h2d(d.edge, st->edge, B * A)) || (rc = h2d(d.time, st->time, B * A)) ||
        (rc = h2d(d.ttl_, st->ttl, B * A)) || (rc = h2d(d.start, st->start, B * A)) ||
        (rc = h2d(d.spw, st->spw, B * A)) || (rc = h2d(d.steps, st->agent_steps, B * A)) ||
        (rc = h2d(d.size, st->size, B * A)) || (rc = h2d(d.visited, st->visited, B * A * 2)) ||
        (rc = h2d(d.amask, st->amask, B * A * 4)) || (rc = h2d(d.load, st->loads, B * E)) ||
        (rc = h2d(d.topo_seed, st->topo_seed, B)) || (rc = h2d(d.topo_reps, st->topo_reps, B)) ||
        (rc = h2d(d.edge_a, st->edge_a, B * E)) || (rc = h2d(d.edge_b, st->edge_b, B * E)) ||
        (rc = h2d(d.edge_len, st->edge_len, B * E)) || (rc = h2d(d.nbr_edge, st->nbr_edge, B * N * 3)) ||
        (rc = h2d(d.seq_index, st->seq_index, B)))
        return rc;
    if (st->nbr_edge) {  // neighbour ids in the per-node edge order (ascending neighbour id)
        std::vector<int32_t> nbr(B * N * 3);
        for (size_t b = 0; b < B; b++)
            for (size_t v = 0; v < N; v++)
                for (int k = 0; k < 3; k++) {
                    const int32_t e = st->nbr_edge[(b * N + v) * 3 + k];
                    nbr[(b * N + v) * 3 + k] =
                        e < 0 ? -1 : (st->edge_a[b * E + e] == (int32_t)v ? st->edge_b[b * E + e] : st->edge_a[b * E + e]);
                }
        GM_HIP(hipMemcpy(d.nbr, nbr.data(), nbr.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    if (st->apsp) {
        std::vector<int16_t> tmp(B * N * N);
        for (size_t i = 0; i < tmp.size(); i++) tmp[i] = (int16_t)st->apsp[i];
        GM_HIP(hipMemcpy(d.apsp, tmp.data(), tmp.size() * sizeof(int16_t), hipMemcpyHostToDevice));
    }
    if (st->rng_key && st->rng_pos) {
        std::vector<uint32_t> mt(B * 2 * MT_N, 0u);
        for (size_t b = 0; b < B; b++) memcpy(mt.data() + b * 2 * MT_N, st->rng_key + b * MT_N, MT_N * 4);
        std::vector<int32_t> zero(B, 0);
        GM_HIP(hipMemcpy(d.mt, mt.data(), mt.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        GM_HIP(hipMemcpy(d.mt_cur, zero.data(), B * sizeof(int32_t), hipMemcpyHostToDevice));
        GM_HIP(hipMemcpy(d.mt_has_next, zero.data(), B * sizeof(int32_t), hipMemcpyHostToDevice));
        GM_HIP(hipMemcpy(d.mt_pos, st->rng_pos, B * sizeof(int32_t), hipMemcpyHostToDevice));
    } else if (st->rng_key || st->rng_pos) {
        return gm_fail(GM_ERR_INVALID_ARG, "gm_env_set_state: rng_key and rng_pos go together");
    }
    return GM_OK;
}

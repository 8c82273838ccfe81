// gm_simple.hip — batched SimpleEnvironment (reference src/env/simple_environment.py:45-334,
// BASELINE config 1) as HIP kernels for gfx950, plus its C ABI.
//
// Three routers on a line, one packet starting at the middle router; action 0/1 picks
// one of the middle router's two edges, the reward is the score (-1/+1) of the router
// reached and the packet returns to the middle. Every draw of the reference's numpy
// stream (scores, positions, edge order) happens in the same order on a per-env
// numpy-legacy MT19937 stream (the same ring as the routing env, gm_device.hpp), so
// traces are bit-exact against the reference for a given seed.
//
// Layout in HBM (library-owned, env-major): score/redge/eend/start/now int32,
// rng u32 [n_env][2][624] + cur/pos/has_next. One 64-lane wave per env for the
// RNG-consuming kernels (reset, ε-greedy), one thread per env for step/observe.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/graph_marl_amd.h"
#include "gm_device.hpp"

using namespace gm;

int gm_fail(int code, const std::string& msg);

struct SimpleDev {
    int n_env, env_var, random_topology;
    int32_t* score;  // [n_env][3]
    int32_t* redge;  // [n_env][3][2] router edge list (-1 = none)
    int32_t* eend;   // [n_env][2][2] edge endpoints (start, end)
    int32_t* start;  // [n_env]
    int32_t* now;    // [n_env]
    uint32_t* mt;
    int32_t *mt_cur, *mt_pos, *mt_has_next;
    int32_t* err;
};

struct gm_simple_env {
    SimpleDev d;
    std::vector<void*> allocs;
    int device;
};

namespace {

constexpr int SN = 3;

__device__ MainRng open_rng(const SimpleDev& d, int env, uint32_t* buf, uint32_t* tmp) {
    MainRng r;
    r.g = d.mt + (size_t)env * 2 * MT_N;
    r.buf = buf;
    r.tmp = tmp;
    r.cur = d.mt_cur[env];
    r.pos = d.mt_pos[env];
    r.has_next = d.mt_has_next[env];
    r.n = 0;
    r.k = 0;
    return r;
}

__device__ void close_rng(const SimpleDev& d, int env, MainRng& r) {
    r.commit();
    if (lane_id() == 0) {
        d.mt_cur[env] = r.cur;
        d.mt_pos[env] = r.pos;
        d.mt_has_next[env] = r.has_next;
    }
}

// RandomState.shuffle of n <= 3 items (legacy: for i = n-1..1, j = random_interval(i))
__device__ __forceinline__ void shuffle(MainRng& r, int* x, int n) {
    for (int i = n - 1; i >= 1; i--) {
        int j = (int)r.randint(i + 1);
        int t = x[i];
        x[i] = x[j];
        x[j] = t;
    }
}

// observation outputs of one env (thread per env)
__device__ void emit(const SimpleDev& d, int env, const gm_simple_obs& o) {
    const int now = d.now[env];
    const int32_t* re = d.redge + (size_t)env * SN * 2;
    const int32_t* ee = d.eend + (size_t)env * 4;
    int adj[SN][SN];
    for (int i = 0; i < SN; i++)
        for (int j = 0; j < SN; j++) adj[i][j] = i == j;
    // router.neighbor lists: the middle router links to both others (simple_environment.py:151-154)
    for (int i = 0; i < SN; i++)
        for (int k = 0; k < 2; k++) {
            int t = re[i * 2 + k];
            if (t < 0) continue;
            int other = ee[t * 2] == i ? ee[t * 2 + 1] : ee[t * 2];
            adj[i][other] = 1;
        }
    if (o.obs) {
        float* ob = o.obs + (size_t)env * o.obs_row_stride;
        ob[0] = (float)now;
        if (d.env_var != 1) {  // [now, adjacency (9), node scores (3)] (simple_environment.py:250-276)
            for (int i = 0; i < SN; i++)
                for (int j = 0; j < SN; j++) ob[1 + i * SN + j] = (float)adj[i][j];
            for (int i = 0; i < SN; i++) ob[1 + SN * SN + i] = (float)d.score[(size_t)env * SN + i];
        }
    }
    if (o.node_obs)
        for (int i = 0; i < SN; i++) o.node_obs[(size_t)env * SN + i] = (float)d.score[(size_t)env * SN + i];
    if (o.node_adj)
        for (int i = 0; i < SN; i++)
            for (int j = 0; j < SN; j++) o.node_adj[(size_t)env * SN * SN + i * SN + j] = (int8_t)adj[i][j];
    if (o.nbr)  // ascending neighbour ids, -1 padded to degree 2
        for (int i = 0; i < SN; i++) {
            int c = 0;
            for (int j = 0; j < SN; j++)
                if (j != i && adj[i][j]) o.nbr[(size_t)env * SN * 2 + i * 2 + c++] = j;
            for (; c < 2; c++) o.nbr[(size_t)env * SN * 2 + i * 2 + c] = -1;
        }
    if (o.agent_node) o.agent_node[env] = now;
}

// SimpleEnvironment._build_network (simple_environment.py:123-209)
__global__ __launch_bounds__(64) void k_simple_reset(SimpleDev d, const uint8_t* mask, gm_simple_obs o) {
    const int env = blockIdx.x;
    if (mask && !mask[env]) {
        if (lane_id() == 0) emit(d, env, o);
        return;
    }
    __shared__ uint32_t rbuf[RNG_BUF];
    __shared__ uint32_t rtmp[MT_N];
    MainRng r = open_rng(d, env, rbuf, rtmp);
    r.prefetch(32);
    const bool rt = d.random_topology != 0;
    int border[2] = {-1, 1};
    shuffle(r, border, 2);
    int sc[3] = {border[0], 0, border[1]};
    if (rt) shuffle(r, sc, 3);
    const int n0 = sc[0] == 0 ? 0 : (sc[1] == 0 ? 1 : 2);
    const int n1 = (n0 + 1) % 3, n2 = (n1 + 1) % 3;
    for (int i = 0; i < 3; i++) {  // Router(x, y): positions only feed the plot
        (void)r.random();
        (void)r.random();
    }
    int dest[2] = {n1, n2};
    if (rt) shuffle(r, dest, 2);
    int e0[2] = {n0, dest[0]};
    if (rt) shuffle(r, e0, 2);
    int e1[2] = {n0, dest[1]};
    if (rt) shuffle(r, e1, 2);
    int order[2] = {0, 1};
    if (rt && dest[1] < dest[0]) {  // sort_edges: np.argsort(edge_destinations)
        order[0] = 1;
        order[1] = 0;
    }
    close_rng(d, env, r);
    if (lane_id() == 0) {
        int32_t* s = d.score + (size_t)env * SN;
        int32_t* re = d.redge + (size_t)env * SN * 2;
        int32_t* ee = d.eend + (size_t)env * 4;
        for (int i = 0; i < 3; i++) s[i] = sc[i];
        for (int i = 0; i < SN * 2; i++) re[i] = -1;
        re[n0 * 2] = order[0];
        re[n0 * 2 + 1] = order[1];
        re[dest[0] * 2] = 0;
        re[dest[1] * 2] = 1;
        ee[0] = e0[0];
        ee[1] = e0[1];
        ee[2] = e1[0];
        ee[3] = e1[1];
        d.start[env] = n0;
        d.now[env] = n0;
        emit(d, env, o);
    }
}

// SimpleEnvironment.step (simple_environment.py:283-315)
__global__ void k_simple_step(SimpleDev d, const int32_t* actions, float* reward, uint8_t* done, gm_simple_obs o) {
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= d.n_env) return;
    const int act = actions[env];
    int now = d.now[env];
    float rw = 0.f;
    const int t = (act == 0 || act == 1) ? d.redge[(size_t)env * SN * 2 + now * 2 + act] : -1;
    if (t < 0) {
        atomicExch(d.err, GM_ERR_INVALID_ARG);
    } else {
        const int32_t* ee = d.eend + (size_t)env * 4;
        now = ee[t * 2] == now ? ee[t * 2 + 1] : ee[t * 2];
        rw = (float)d.score[(size_t)env * SN + now];
    }
    if (reward) reward[env] = rw;
    if (done) done[env] = 1;
    d.now[env] = d.start[env];
    emit(d, env, o);
}

__global__ void k_simple_observe(SimpleDev d, gm_simple_obs o) {
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env < d.n_env) emit(d, env, o);
}

// EpsilonGreedy.__call__ (src/policy.py:44-50) with action_space 2 and one agent:
// randint(2, size=1) then rand(1) from the env's stream, first-maximum argmax.
__global__ __launch_bounds__(64) void k_simple_egreedy(SimpleDev d, const float* q, double eps, int32_t* actions) {
    const int env = blockIdx.x;
    __shared__ uint32_t rbuf[RNG_BUF];
    __shared__ uint32_t rtmp[MT_N];
    MainRng r = open_rng(d, env, rbuf, rtmp);
    r.prefetch(3);
    const int ra = (int)(r.next32() & 1u);
    const double u = r.random();
    close_rng(d, env, r);
    if (lane_id() == 0) {
        const float q0 = q[(size_t)env * 2], q1 = q[(size_t)env * 2 + 1];
        const int best = q1 > q0 ? 1 : 0;
        actions[env] = u < eps ? ra : best;
    }
}

__global__ void k_simple_seed(SimpleDev d, const uint32_t* seeds) {
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
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
}

int launched() {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return gm_fail(GM_ERR_HIP, std::string("kernel launch: ") + hipGetErrorString(e));
    return GM_OK;
}

unsigned blocks(int n) { return (unsigned)((n + 127) / 128); }

}  // namespace

#define SIM_HIP(call)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return gm_fail(GM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" int gm_simple_destroy(gm_simple_env* env) {
    if (!env) return GM_OK;
    (void)hipSetDevice(env->device);
    for (void* p : env->allocs) (void)hipFree(p);
    delete env;
    return GM_OK;
}

extern "C" int gm_simple_create(int32_t n_env, int32_t env_var, int32_t random_topology, const uint32_t* seeds,
                                int32_t device, gm_simple_env** out) {
    if (!out || !seeds || n_env <= 0 || env_var < 1 || env_var > 3)
        return gm_fail(GM_ERR_INVALID_ARG, "gm_simple_create: bad arguments");
    *out = nullptr;
    SIM_HIP(hipSetDevice(device));
    gm_simple_env* env = new gm_simple_env();
    env->device = device;
    SimpleDev& d = env->d;
    d.n_env = n_env;
    d.env_var = env_var;
    d.random_topology = random_topology;
    const size_t B = n_env;
#define ALLOC(ptr, count)                                                                   \
    do {                                                                                    \
        void* p_ = nullptr;                                                                 \
        if (hipMalloc(&p_, (count) * sizeof(*(ptr))) != hipSuccess) {                      \
            gm_simple_destroy(env);                                                         \
            return gm_fail(GM_ERR_OOM, "gm_simple_create: hipMalloc failed");               \
        }                                                                                   \
        env->allocs.push_back(p_);                                                          \
        ptr = reinterpret_cast<decltype(ptr)>(p_);                                          \
    } while (0)
    ALLOC(d.score, B * SN);
    ALLOC(d.redge, B * SN * 2);
    ALLOC(d.eend, B * 4);
    ALLOC(d.start, B);
    ALLOC(d.now, B);
    ALLOC(d.mt, B * 2 * MT_N);
    ALLOC(d.mt_cur, B);
    ALLOC(d.mt_pos, B);
    ALLOC(d.mt_has_next, B);
    ALLOC(d.err, 1);
    uint32_t* seeds_d = nullptr;
    ALLOC(seeds_d, B);
#undef ALLOC
    SIM_HIP(hipMemcpy(seeds_d, seeds, B * sizeof(uint32_t), hipMemcpyHostToDevice));
    SIM_HIP(hipMemset(d.err, 0, sizeof(int32_t)));
    SIM_HIP(hipMemset(d.redge, 0xff, B * SN * 2 * sizeof(int32_t)));
    SIM_HIP(hipMemset(d.eend, 0, B * 4 * sizeof(int32_t)));
    SIM_HIP(hipMemset(d.score, 0, B * SN * sizeof(int32_t)));
    SIM_HIP(hipMemset(d.start, 0, B * sizeof(int32_t)));
    SIM_HIP(hipMemset(d.now, 0, B * sizeof(int32_t)));
    hipLaunchKernelGGL(k_simple_seed, dim3(blocks(n_env)), dim3(128), 0, 0, d, seeds_d);
    int rc = launched();
    if (rc != GM_OK) {
        gm_simple_destroy(env);
        return rc;
    }
    SIM_HIP(hipDeviceSynchronize());
    *out = env;
    return GM_OK;
}

static int check_obs(const gm_simple_env* env, const gm_simple_obs* o) {
    if (o && o->obs && o->obs_row_stride < (env->d.env_var == 1 ? 1 : 13))
        return gm_fail(GM_ERR_INVALID_ARG, "gm_simple: obs_row_stride smaller than the observation size");
    return GM_OK;
}

extern "C" int gm_simple_reset(gm_simple_env* env, const uint8_t* reset_mask, const gm_simple_obs* obs,
                               void* stream) {
    if (!env) return gm_fail(GM_ERR_INVALID_ARG, "null env");
    if (int rc = check_obs(env, obs)) return rc;
    gm_simple_obs o = obs ? *obs : gm_simple_obs{};
    hipLaunchKernelGGL(k_simple_reset, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, reset_mask, o);
    return launched();
}

extern "C" int gm_simple_step(gm_simple_env* env, const int32_t* actions, float* reward, uint8_t* done,
                              const gm_simple_obs* obs, void* stream) {
    if (!env || !actions) return gm_fail(GM_ERR_INVALID_ARG, "gm_simple_step: null argument");
    if (int rc = check_obs(env, obs)) return rc;
    gm_simple_obs o = obs ? *obs : gm_simple_obs{};
    hipLaunchKernelGGL(k_simple_step, dim3(blocks(env->d.n_env)), dim3(128), 0, (hipStream_t)stream, env->d, actions,
                       reward, done, o);
    return launched();
}

extern "C" int gm_simple_observe(gm_simple_env* env, const gm_simple_obs* obs, void* stream) {
    if (!env || !obs) return gm_fail(GM_ERR_INVALID_ARG, "gm_simple_observe: null argument");
    if (int rc = check_obs(env, obs)) return rc;
    hipLaunchKernelGGL(k_simple_observe, dim3(blocks(env->d.n_env)), dim3(128), 0, (hipStream_t)stream, env->d, *obs);
    return launched();
}

extern "C" int gm_simple_policy_egreedy(gm_simple_env* env, const float* q, double epsilon, int32_t* actions,
                                        void* stream) {
    if (!env || !q || !actions) return gm_fail(GM_ERR_INVALID_ARG, "gm_simple_policy_egreedy: null argument");
    hipLaunchKernelGGL(k_simple_egreedy, dim3(env->d.n_env), dim3(64), 0, (hipStream_t)stream, env->d, q, epsilon,
                       actions);
    return launched();
}

extern "C" int gm_simple_get_state(gm_simple_env* env, gm_simple_state* st) {
    if (!env || !st) return gm_fail(GM_ERR_INVALID_ARG, "null argument");
    SIM_HIP(hipSetDevice(env->device));
    SIM_HIP(hipDeviceSynchronize());
    const SimpleDev& d = env->d;
    int32_t err = 0;
    SIM_HIP(hipMemcpy(&err, d.err, sizeof(err), hipMemcpyDeviceToHost));
    if (err) {
        SIM_HIP(hipMemset(d.err, 0, sizeof(int32_t)));
        return gm_fail(err, "gm_simple: an action outside {0, 1} was stepped");
    }
    const size_t B = d.n_env;
    if (st->score) SIM_HIP(hipMemcpy(st->score, d.score, B * SN * 4, hipMemcpyDeviceToHost));
    if (st->router_edge) SIM_HIP(hipMemcpy(st->router_edge, d.redge, B * SN * 2 * 4, hipMemcpyDeviceToHost));
    if (st->edge_end) SIM_HIP(hipMemcpy(st->edge_end, d.eend, B * 4 * 4, hipMemcpyDeviceToHost));
    if (st->start) SIM_HIP(hipMemcpy(st->start, d.start, B * 4, hipMemcpyDeviceToHost));
    if (st->now) SIM_HIP(hipMemcpy(st->now, d.now, B * 4, hipMemcpyDeviceToHost));
    return GM_OK;
}

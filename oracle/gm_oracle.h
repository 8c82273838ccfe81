/* gm_oracle.h — CPU restatement of graph-marl's routing environment.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity checker (and the CPU-baseline
 * "port" in bench.py), never the product path. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it.
 *
 * Parity pinned: checked against golden vectors produced by importing the
 * reference (tests/golden/make_golden.py) — numpy legacy RNG streams, topologies,
 * and full environment traces.
 */
#ifndef GM_ORACLE_H
#define GM_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#define GMO_MAXN 128
#define GMO_MAXE (GMO_MAXN * 3 / 2)
#define GMO_MAXA 256

typedef struct {
    uint32_t key[624];
    int32_t pos;
} gmo_mt;

void gmo_mt_seed(gmo_mt* s, uint32_t seed);
uint32_t gmo_mt_next32(gmo_mt* s);
double gmo_mt_random(gmo_mt* s);
int64_t gmo_mt_randint(gmo_mt* s, int64_t high);

typedef struct {
    int32_t n, n_edges;
    double x[GMO_MAXN], y[GMO_MAXN];
    int32_t deg[GMO_MAXN];
    int32_t neighbors[GMO_MAXN][3];  /* insertion order */
    int32_t node_edges[GMO_MAXN][3]; /* sorted by neighbour id */
    int32_t nbr[GMO_MAXN][3];        /* neighbour ids, ascending */
    int32_t edge_a[GMO_MAXE], edge_b[GMO_MAXE], edge_len[GMO_MAXE];
    int32_t apsp[GMO_MAXN][GMO_MAXN];
    int64_t seed;
    int32_t repetitions;
} gmo_topo;

/* topology modes (mirror Network's seed handling, src/env/network.py:215-272, 356-371) */
enum { GMO_TOPO_FIXED = 0, GMO_TOPO_RANDOM = 1, GMO_TOPO_LIST = 2, GMO_TOPO_SEQUENTIAL = 3 };

typedef struct {
    int32_t n_nodes, n_data;
    int32_t congestion, action_mask, ttl;
    int32_t topo_mode;
    int64_t topo_seed;             /* FIXED */
    const int64_t* seed_list;      /* LIST / SEQUENTIAL */
    int32_t n_seed_list;
    const int64_t* excluded;       /* sorted ascending, may be NULL */
    int32_t n_excluded;
    int32_t env_var;               /* 1 INDEPENDENT, 2 WITH_K_NEIGHBORS, 3 GLOBAL (0 = 1) */
    int32_t k;                     /* neighbours in variant-2 observations (routing.py:59, default 3) */
} gmo_config;

typedef struct {
    gmo_config cfg;
    gmo_mt rng;
    gmo_topo topo;
    int32_t seq_index;
    int32_t now[GMO_MAXA], target[GMO_MAXA], edge[GMO_MAXA], time[GMO_MAXA], ttl[GMO_MAXA];
    int32_t start[GMO_MAXA], spw[GMO_MAXA];
    double size[GMO_MAXA];
    uint64_t visited[GMO_MAXA][2];
    double agent_steps[GMO_MAXA];
    double load[GMO_MAXE];
    uint8_t amask[GMO_MAXA][4];
    /* neighbour lists from the last observation (for the agent adjacency) */
    int32_t neigh_cnt[GMO_MAXA];
    int16_t neigh[GMO_MAXA][GMO_MAXA];
} gmo_env;

typedef struct {
    double looped;
    int32_t throughput, dropped, blocked;
    int32_t n_delays, n_arrived;
    double delays[GMO_MAXA], delays_arrived[GMO_MAXA], spr[GMO_MAXA];
} gmo_info;

int gmo_topo_attempt(gmo_topo* t, int32_t n, gmo_mt* rng);
int gmo_topo_valid(const gmo_topo* t);
void gmo_topo_apsp(gmo_topo* t);
int64_t gmo_create_valid(gmo_topo* t, const gmo_config* c, gmo_mt* main_rng, int32_t seed_index);
int gmo_build_seed_list(int32_t n, int64_t init_seed, int32_t count, const int64_t* excl, int32_t n_excl, int64_t* out);

void gmo_env_init(gmo_env* e, const gmo_config* c, uint32_t seed);
void gmo_env_reset(gmo_env* e);
void gmo_env_step(gmo_env* e, const int32_t* act, float* reward, uint8_t* done, gmo_info* info);
void gmo_env_observe(gmo_env* e, float* obs, float* node_obs, int8_t* adj, int8_t* node_agent, float* aux);
void gmo_env_final_delays(const gmo_env* e, double* out, int32_t* n_out);
int32_t gmo_obs_dim(int32_t n);
/* agent observation width of a configuration: 6N+10 (+5k for variant 2, +N^2+N(4N+8) for 3) */
int32_t gmo_obs_dim_cfg(const gmo_config* c);
int32_t gmo_node_obs_dim(int32_t n);
size_t gmo_env_sizeof(void);

/* CPU baseline: run n_env independent envs for `steps` steps with uniform random
 * actions (action tape from a splitmix stream), OpenMP over envs. Returns seconds. */
double gmo_bench_rollout(const gmo_config* c, int32_t n_env, int32_t steps, int32_t episode_steps,
                         int32_t n_threads, float* obs_out, float* node_obs_out);
/* batched CPU-baseline driver (OpenMP over envs) */
gmo_env* gmo_batch_create(const gmo_config* c, int32_t n_env, uint32_t seed_base);
void gmo_batch_free(gmo_env* envs);
void gmo_batch_run(gmo_env* envs, int32_t n_env, int32_t do_reset, const int32_t* act, float* reward, uint8_t* done,
                   float* obs, int64_t obs_stride, float* node_obs, int32_t* agent_node, int32_t* nbr);
#endif

/* gm_oracle.c — plain-C restatement of graph-marl's routing environment.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU-baseline "port"); see gm_oracle.h.
 * Every function cites the reference file:line it restates (paths relative to the
 * reference repository root). Compile with -ffp-contract=off: the reference
 * evaluates every floating-point expression with separate IEEE roundings.
 */
#include "gm_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------------------
 * numpy legacy RandomState (MT19937). The reference draws every random number
 * through np.random.* (src/env/routing.py:130-134, src/env/network.py:136,230-255,
 * src/policy.py:46-47). Seeding = init_genrand (numpy _legacy_seeding),
 * randint = masked rejection on 32-bit draws, random() = 53-bit double.
 * ------------------------------------------------------------------------- */
void gmo_mt_seed(gmo_mt* s, uint32_t seed) {
    s->key[0] = seed;
    for (int i = 1; i < 624; i++)
        s->key[i] = 1812433253u * (s->key[i - 1] ^ (s->key[i - 1] >> 30)) + (uint32_t)i;
    s->pos = 624;
}

static void mt_gen(gmo_mt* s) {
    uint32_t* k = s->key;
    int i;
    uint32_t y;
    for (i = 0; i < 624 - 397; i++) {
        y = (k[i] & 0x80000000u) | (k[i + 1] & 0x7fffffffu);
        k[i] = k[i + 397] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    for (; i < 623; i++) {
        y = (k[i] & 0x80000000u) | (k[i + 1] & 0x7fffffffu);
        k[i] = k[i + (397 - 624)] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    }
    y = (k[623] & 0x80000000u) | (k[0] & 0x7fffffffu);
    k[623] = k[396] ^ (y >> 1) ^ (-(y & 1u) & 0x9908b0dfu);
    s->pos = 0;
}

uint32_t gmo_mt_next32(gmo_mt* s) {
    if (s->pos == 624) mt_gen(s);
    uint32_t y = s->key[s->pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

double gmo_mt_random(gmo_mt* s) {
    int32_t a = (int32_t)(gmo_mt_next32(s) >> 5), b = (int32_t)(gmo_mt_next32(s) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

int64_t gmo_mt_randint(gmo_mt* s, int64_t high) {
    uint64_t rng = (uint64_t)(high - 1);
    if (rng == 0) return 0;
    uint32_t mask = (uint32_t)rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = (gmo_mt_next32(s) & mask)) > (uint32_t)rng) {
    }
    return (int64_t)v;
}

/* ---------------------------------------------------------------------------
 * Topology (src/env/network.py:122-195 _create_random_topology)
 * ------------------------------------------------------------------------- */
int gmo_topo_attempt(gmo_topo* t, int32_t n, gmo_mt* rng) {
    t->n = n;
    t->n_edges = 0;
    for (int i = 0; i < n; i++) { /* network.py:134-138: x then y per node */
        t->x[i] = gmo_mt_random(rng);
        t->y[i] = gmo_mt_random(rng);
        t->deg[i] = 0;
    }
    double d2[GMO_MAXN];
    int32_t order[GMO_MAXN];
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) { /* network.py:143-150 */
            double dx = t->x[j] - t->x[i], dy = t->y[j] - t->y[i];
            double a = dx * dx, b = dy * dy;
            d2[j] = a + b;
        }
        /* stable sort by distance (network.py:153; list.sort is stable) */
        for (int j = 0; j < n; j++) order[j] = j;
        for (int j = 1; j < n; j++) {
            int32_t v = order[j];
            int k = j - 1;
            while (k >= 0 && d2[order[k]] > d2[v]) {
                order[k + 1] = order[k];
                k--;
            }
            order[k + 1] = v;
        }
        for (int r = 1; r < n; r++) { /* network.py:157-188 */
            if (t->deg[i] == 3) break;
            int32_t c = order[r];
            int linked = 0;
            for (int q = 0; q < t->deg[c]; q++) linked |= (t->neighbors[c][q] == i);
            if (t->deg[c] < 3 && !linked) {
                t->neighbors[i][t->deg[i]] = c;
                t->neighbors[c][t->deg[c]] = i;
                double sq = sqrt(d2[c]);
                double s10 = sq * 10.0;
                int32_t k10 = (int32_t)s10;
                int32_t len = k10 / 2 + 1; /* int(int(sqrt*10)/2 + 1), network.py:173 */
                int32_t e = t->n_edges++;
                t->edge_a[e] = i < c ? i : c;
                t->edge_b[e] = i < c ? c : i;
                t->edge_len[e] = len;
                t->node_edges[c][t->deg[c]] = e; /* candidate first, network.py:180-181 */
                t->node_edges[i][t->deg[i]] = e;
                t->deg[c]++;
                t->deg[i]++;
            }
        }
    }
    /* order router edges by neighbour node id (network.py:191-195) */
    for (int i = 0; i < n; i++) {
        int d = t->deg[i];
        for (int a = 1; a < d; a++) {
            int32_t e = t->node_edges[i][a];
            int32_t oe = t->edge_a[e] == i ? t->edge_b[e] : t->edge_a[e];
            int b = a - 1;
            while (b >= 0) {
                int32_t eb = t->node_edges[i][b];
                int32_t ob = t->edge_a[eb] == i ? t->edge_b[eb] : t->edge_a[eb];
                if (ob <= oe) break;
                t->node_edges[i][b + 1] = eb;
                b--;
            }
            t->node_edges[i][b + 1] = e;
        }
        for (int a = 0; a < d; a++) {
            int32_t e = t->node_edges[i][a];
            t->nbr[i][a] = t->edge_a[e] == i ? t->edge_b[e] : t->edge_a[e];
        }
    }
    return 0;
}

/* src/env/network.py:197-213: every node has 3 neighbours and the graph is connected */
int gmo_topo_valid(const gmo_topo* t) {
    int n = t->n;
    for (int i = 0; i < n; i++)
        if (t->deg[i] < 3) return 0;
    uint8_t seen[GMO_MAXN] = {0};
    int32_t stack[GMO_MAXN], sp = 0, cnt = 1;
    seen[0] = 1;
    stack[sp++] = 0;
    while (sp) {
        int v = stack[--sp];
        for (int q = 0; q < t->deg[v]; q++) {
            int u = t->neighbors[v][q];
            if (!seen[u]) {
                seen[u] = 1;
                cnt++;
                stack[sp++] = u;
            }
        }
    }
    return cnt == n;
}

/* src/env/network.py:274-290: only the path *weights* are consumed by the env
 * (routing.py:137,250), which any exact APSP reproduces. */
void gmo_topo_apsp(gmo_topo* t) {
    int n = t->n;
    const int32_t INF = 1 << 28;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) t->apsp[i][j] = i == j ? 0 : INF;
    for (int e = 0; e < t->n_edges; e++) {
        int a = t->edge_a[e], b = t->edge_b[e];
        if (t->edge_len[e] < t->apsp[a][b]) t->apsp[a][b] = t->apsp[b][a] = t->edge_len[e];
    }
    for (int k = 0; k < n; k++)
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                int32_t v = t->apsp[i][k] + t->apsp[k][j];
                if (v < t->apsp[i][j]) t->apsp[i][j] = v;
            }
}

static int is_excluded(const int64_t* ex, int32_t n, int64_t s) {
    int32_t lo = 0, hi = n - 1;
    while (lo <= hi) {
        int32_t m = (lo + hi) / 2;
        if (ex[m] == s) return 1;
        if (ex[m] < s) lo = m + 1; else hi = m - 1;
    }
    return 0;
}

static int64_t draw_seed(gmo_mt* r, const int64_t* ex, int32_t nex) {
    int64_t s = gmo_mt_randint(r, 2147483647LL);
    while (ex && is_excluded(ex, nex, s)) s = gmo_mt_randint(r, 2147483647LL);
    return s;
}

/* src/env/network.py:215-272 _create_valid_network. seed_index >= 0 selects from the
 * list without drawing (sequential mode, network.py:234-235). The caller's main
 * stream is only touched by the seed choice (state restored, network.py:241,258). */
int64_t gmo_create_valid(gmo_topo* t, const gmo_config* c, gmo_mt* main_rng, int32_t seed_index) {
    int no_seed = !(c->topo_mode == GMO_TOPO_FIXED || c->topo_mode == GMO_TOPO_LIST ||
                    c->topo_mode == GMO_TOPO_SEQUENTIAL);
    int64_t seed;
    if (no_seed) {
        seed = draw_seed(main_rng, c->excluded, c->n_excluded);
    } else if (c->topo_mode == GMO_TOPO_FIXED) {
        seed = c->topo_seed; /* np.random.choice of a 1-element list draws nothing */
    } else if (seed_index >= 0) {
        seed = c->seed_list[seed_index];
    } else {
        seed = c->seed_list[gmo_mt_randint(main_rng, c->n_seed_list)];
    }
    gmo_mt topo_rng;
    gmo_mt_seed(&topo_rng, (uint32_t)seed);
    t->repetitions = 0;
    for (;;) {
        gmo_topo_attempt(t, c->n_nodes, &topo_rng);
        t->repetitions++;
        if (gmo_topo_valid(t)) break;
        if (!no_seed || t->repetitions > 100000) { /* reference asserts (network.py:251) */
            t->seed = -1;
            return -1;
        }
        seed = draw_seed(&topo_rng, c->excluded, c->n_excluded);
        gmo_mt_seed(&topo_rng, (uint32_t)seed);
    }
    gmo_topo_apsp(t);
    t->seed = seed;
    return seed;
}

/* src/env/network.py:100-120 build_seed_list (unique valid seeds from init seed) */
int gmo_build_seed_list(int32_t n, int64_t init_seed, int32_t count, const int64_t* excl, int32_t n_excl,
                        int64_t* out) {
    gmo_config c;
    memset(&c, 0, sizeof(c));
    c.n_nodes = n;
    c.topo_mode = GMO_TOPO_RANDOM;
    c.excluded = excl;
    c.n_excluded = n_excl;
    gmo_mt r;
    gmo_mt_seed(&r, (uint32_t)init_seed);
    gmo_topo* t = (gmo_topo*)malloc(sizeof(gmo_topo));
    int32_t have = 0;
    while (have < count) {
        int64_t s = gmo_create_valid(t, &c, &r, -1);
        int dup = 0;
        for (int i = 0; i < have; i++) dup |= out[i] == s;
        if (!dup) out[have++] = s;
    }
    free(t);
    return have;
}

/* ---------------------------------------------------------------------------
 * Routing environment (src/env/routing.py)
 * ------------------------------------------------------------------------- */
static inline int other_node(const gmo_topo* t, int e, int v) {
    return t->edge_a[e] == v ? t->edge_b[e] : t->edge_a[e];
}
static inline int vis_has(const uint64_t* v, int i) { return (int)((v[i >> 6] >> (i & 63)) & 1u); }
static inline void vis_add(uint64_t* v, int i) { v[i >> 6] |= 1ull << (i & 63); }

int32_t gmo_obs_dim(int32_t n) { return 6 * n + 10; }
/* routing.py:268-358: variant 2 appends k x (now, target, edge, size, own id) of the first k
 * packets on the same or an adjacent node, variant 3 the flattened I+A and node observations */
int32_t gmo_obs_dim_cfg(const gmo_config* c) {
    int32_t n = c->n_nodes, d = 6 * n + 10;
    if (c->env_var == 2) d += 5 * (c->k > 0 ? c->k : 0);
    if (c->env_var == 3) d += n * n + n * (4 * n + 8);
    return d;
}
int32_t gmo_node_obs_dim(int32_t n) { return 4 * n + 8; }
size_t gmo_env_sizeof(void) { return sizeof(gmo_env); }

void gmo_env_init(gmo_env* e, const gmo_config* c, uint32_t seed) {
    memset(e, 0, sizeof(*e));
    e->cfg = *c;
    gmo_mt_seed(&e->rng, seed);
    e->seq_index = 0;
}

/* src/env/routing.py:119-144 reset_packet */
static void reset_packet(gmo_env* e, int i) {
    gmo_topo* t = &e->topo;
    if (e->edge[i] != -1) e->load[e->edge[i]] -= e->size[i];
    int32_t start = (int32_t)gmo_mt_randint(&e->rng, t->n);
    int32_t target = (int32_t)gmo_mt_randint(&e->rng, t->n);
    double size = gmo_mt_random(&e->rng);
    e->now[i] = start;
    e->target[i] = target;
    e->size[i] = size;
    e->start[i] = start;
    e->time[i] = 0;
    e->edge[i] = -1;
    e->ttl[i] = e->cfg.ttl;
    e->spw[i] = t->apsp[start][target];
    e->visited[i][0] = e->visited[i][1] = 0;
    vis_add(e->visited[i], start);
    if (e->cfg.action_mask) {
        memset(e->amask[i], 0, 4);
        e->amask[i][0] = start != target;
    }
}

/* src/env/routing.py:160-178 reset (+ network.py:366-371) */
void gmo_env_reset(gmo_env* e) {
    int32_t seed_index = -1;
    const gmo_config* c = &e->cfg;
    if (c->topo_mode == GMO_TOPO_SEQUENTIAL && c->n_seed_list > 1) { /* network.py:356-364 */
        seed_index = e->seq_index;
        e->seq_index = (seed_index + 1) % c->n_seed_list;
    } else if (c->topo_mode == GMO_TOPO_SEQUENTIAL) {
        seed_index = 0;
    }
    gmo_create_valid(&e->topo, c, &e->rng, seed_index);
    for (int i = 0; i < c->n_data; i++) e->agent_steps[i] = 0.0;
    for (int k = 0; k < e->topo.n_edges; k++) e->load[k] = 0.0;
    for (int i = 0; i < c->n_data; i++) {
        e->edge[i] = -1;
        reset_packet(e, i);
    }
}

/* src/env/routing.py:360-520 step */
void gmo_env_step(gmo_env* e, const int32_t* act, float* reward, uint8_t* done, gmo_info* info) {
    const gmo_config* c = &e->cfg;
    gmo_topo* t = &e->topo;
    int A = c->n_data;
    uint8_t drop[GMO_MAXA], success[GMO_MAXA];
    memset(info, 0, sizeof(*info));
    for (int i = 0; i < A; i++) {
        reward[i] = 0.0f;
        done[i] = 0;
        drop[i] = 0;
        success[i] = 0;
        e->agent_steps[i] += 1.0; /* routing.py:371 */
    }
    /* phase 1: actions in packet-id order (routing.py:380-412) */
    for (int i = 0; i < A; i++) {
        if (e->edge[i] == -1 && act[i] != 0) {
            int te = t->node_edges[e->now[i]][act[i] - 1];
            if (c->congestion && e->load[te] + e->size[i] > 1.0) {
                reward[i] = reward[i] - 0.2f;
                info->blocked++;
            } else {
                e->edge[i] = te;
                e->time[i] = t->edge_len[te];
                e->load[te] += e->size[i];
                e->now[i] = other_node(t, te, e->now[i]);
                if (vis_has(e->visited[i], e->now[i])) info->looped += 1.0;
                else vis_add(e->visited[i], e->now[i]);
            }
        }
    }
    /* phase 2: in-flight packets, arrivals, drops, respawn (routing.py:444-495) */
    for (int i = 0; i < A; i++) {
        e->ttl[i] -= 1;
        if (e->edge[i] != -1) {
            e->time[i] -= 1;
            if (e->time[i] <= 0) {
                e->load[e->edge[i]] -= e->size[i];
                e->edge[i] = -1;
            }
        }
        drop[i] = drop[i] || (c->ttl > 0 && e->ttl[i] <= 0);
        if (c->action_mask) {
            if (e->edge[i] != -1) {
                memset(e->amask[i], 0, 4);
            } else {
                e->amask[i][0] = 1;
                int s = 1;
                for (int k = 0; k < 3; k++) {
                    int o = t->nbr[e->now[i]][k];
                    e->amask[i][1 + k] = (uint8_t)vis_has(e->visited[i], o);
                    s += e->amask[i][1 + k];
                }
                if (s == 4) drop[i] = 1;
            }
        }
        int reached = e->edge[i] == -1 && e->now[i] == e->target[i];
        if (reached || drop[i]) {
            reward[i] = reward[i] + (reached ? 10.0f : -10.0f);
            done[i] = 1;
            success[i] = (uint8_t)reached;
            int32_t opt = e->spw[i] > 1 ? e->spw[i] : 1;
            if (reached) {
                info->delays_arrived[info->n_arrived++] = e->agent_steps[i];
                info->spr[info->n_arrived - 1] = e->agent_steps[i] / (double)opt;
            }
            info->delays[info->n_delays++] = e->agent_steps[i];
            e->agent_steps[i] = 0.0;
            reset_packet(e, i);
        }
    }
    for (int i = 0; i < A; i++) {
        info->throughput += success[i];
        info->dropped += done[i] && !success[i];
    }
}

/* src/env/routing.py:541-546 get_final_info: non-zero agent steps appended to delays */
void gmo_env_final_delays(const gmo_env* e, double* out, int32_t* n_out) {
    int32_t k = 0;
    for (int i = 0; i < e->cfg.n_data; i++)
        if (e->agent_steps[i] != 0.0) out[k++] = e->agent_steps[i];
    *n_out = k;
}

/* Observations:
 *   agent obs   src/env/routing.py:269-358 (_get_observation, INDEPENDENT variant)
 *   agent adj   src/env/routing.py:522-539 (_get_data_adjacency; neigh from 317-327)
 *   node obs    src/env/routing.py:187-235 (get_node_observation)
 *   node-agent  src/env/routing.py:256-267
 *   node aux    src/env/routing.py:237-254
 * Any output pointer may be NULL. */
/* node observation rows (routing.py:187-235): one-hot id, packets waiting (not on an edge)
 * and the sum of their sizes in id order, then per neighbour (ascending id) one-hot, length,
 * load */
static void node_obs_rows(const gmo_env* e, float* node_obs) {
    const gmo_topo* t = &e->topo;
    int n = t->n, A = e->cfg.n_data, ND = gmo_node_obs_dim(n);
    for (int j = 0; j < n; j++) {
        float* o = node_obs + (size_t)j * ND;
        memset(o, 0, sizeof(float) * ND);
        o[j] = 1.0f;
        int np = 0;
        double tl = 0.0;
        for (int i = 0; i < A; i++)
            if (e->now[i] == j && e->edge[i] == -1) {
                np++;
                tl += e->size[i];
            }
        o[n] = (float)np;
        o[n + 1] = (float)tl;
        for (int k = 0; k < 3; k++) {
            int ed = t->node_edges[j][k];
            float* ok = o + n + 2 + k * (n + 2);
            ok[other_node(t, ed, j)] = 1.0f;
            ok[n] = (float)t->edge_len[ed];
            ok[n + 1] = (float)e->load[ed];
        }
    }
}

void gmo_env_observe(gmo_env* e, float* obs, float* node_obs, int8_t* adj, int8_t* node_agent, float* aux) {
    gmo_topo* t = &e->topo;
    int n = t->n, A = e->cfg.n_data;
    int D = gmo_obs_dim_cfg(&e->cfg), D1 = gmo_obs_dim(n), ND = gmo_node_obs_dim(n);
    int var = e->cfg.env_var, K = e->cfg.k;
    float* glob = NULL; /* variant 3: [I+A flattened | node obs flattened] (routing.py:271-274) */
    if (obs && var == 3) {
        glob = (float*)calloc((size_t)n * n + (size_t)n * ND, sizeof(float));
        for (int j = 0; j < n; j++) {
            glob[(size_t)j * n + j] = 1.0f;
            for (int k = 0; k < t->deg[j]; k++) glob[(size_t)j * n + t->neighbors[j][k]] = 1.0f;
        }
        node_obs_rows(e, glob + (size_t)n * n);
    }
    for (int i = 0; i < A; i++) {
        int now = e->now[i];
        if (obs) {
            float* o = obs + (size_t)i * D;
            memset(o, 0, sizeof(float) * D);
            o[now] = 1.0f;
            o[n + e->target[i]] = 1.0f;
            o[2 * n] = (float)(e->edge[i] != -1);
            if (e->edge[i] != -1) o[2 * n + 1 + other_node(t, e->edge[i], now)] = 1.0f;
            o[3 * n + 1] = (float)e->time[i];
            o[3 * n + 2] = (float)e->size[i];
            o[3 * n + 3] = (float)i;
            for (int k = 0; k < 3; k++) {
                int ed = t->node_edges[now][k];
                float* ok = o + 3 * n + 4 + k * (n + 2);
                ok[other_node(t, ed, now)] = 1.0f;
                ok[n] = (float)t->edge_len[ed];
                ok[n + 1] = (float)e->load[ed];
            }
        }
        /* neighbour list: self, then packets on the same or an adjacent node (routing.py:317-327) */
        int cnt = 0, kn = 0;
        e->neigh[i][cnt++] = (int16_t)i;
        for (int j = 0; j < A; j++) {
            if (j == i) continue;
            int nj = e->now[j];
            int adjacent = nj == now;
            for (int k = 0; k < t->deg[now]; k++) adjacent |= t->neighbors[now][k] == nj;
            if (adjacent) {
                e->neigh[i][cnt++] = (int16_t)j;
                if (obs && var == 2 && kn < K) { /* routing.py:329-338 (appends its own id) */
                    float* ok = obs + (size_t)i * D + D1 + 5 * kn;
                    ok[0] = (float)e->now[j];
                    ok[1] = (float)e->target[j];
                    ok[2] = (float)e->edge[j];
                    ok[3] = (float)e->size[j];
                    ok[4] = (float)i;
                    kn++;
                }
            }
        }
        if (obs && var == 2)
            for (int q = 5 * kn; q < 5 * K; q++) obs[(size_t)i * D + D1 + q] = -1.0f; /* placeholders (340-342) */
        if (obs && var == 3) memcpy(obs + (size_t)i * D + D1, glob, sizeof(float) * (size_t)(D - D1));
        e->neigh_cnt[i] = cnt;
    }
    free(glob);
    if (adj) {
        memset(adj, 0, (size_t)A * A);
        for (int i = 0; i < A; i++) {
            adj[(size_t)i * A + i] = 1;
            for (int q = 0; q < e->neigh_cnt[i]; q++) adj[(size_t)i * A + e->neigh[i][q]] = 1;
        }
    }
    if (node_obs) node_obs_rows(e, node_obs);
    if (node_agent) {
        memset(node_agent, 0, (size_t)n * A);
        for (int a = 0; a < A; a++) node_agent[(size_t)e->now[a] * A + a] = 1;
    }
    if (aux) {
        for (int j = 0; j < n; j++)
            for (int k = 0; k < n; k++) aux[(size_t)j * n + k] = (float)t->apsp[j][k];
    }
}

/* ---------------------------------------------------------------------------
 * CPU baseline driver: independent envs, uniform random actions, OpenMP.
 * ------------------------------------------------------------------------- */
static inline uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

double gmo_bench_rollout(const gmo_config* c, int32_t n_env, int32_t steps, int32_t episode_steps,
                         int32_t n_threads, float* obs_out, float* node_obs_out) {
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#endif
    gmo_env* envs = (gmo_env*)malloc(sizeof(gmo_env) * (size_t)n_env);
    int n = c->n_nodes, A = c->n_data;
    size_t D = (size_t)gmo_obs_dim(n), ND = (size_t)gmo_node_obs_dim(n);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < n_env; b++) {
        gmo_env_init(&envs[b], c, (uint32_t)(1000 + b));
        gmo_env_reset(&envs[b]);
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < n_env; b++) {
        gmo_env* e = &envs[b];
        uint64_t sm = 0x1234ull + (uint64_t)b;
        int32_t act[GMO_MAXA];
        float rew[GMO_MAXA];
        uint8_t done[GMO_MAXA];
        gmo_info info;
        for (int s = 0; s < steps; s++) {
            for (int i = 0; i < A; i++) act[i] = (int32_t)(splitmix(&sm) & 3u);
            gmo_env_step(e, act, rew, done, &info);
            if (episode_steps > 0 && (s + 1) % episode_steps == 0) gmo_env_reset(e);
            gmo_env_observe(e, obs_out ? obs_out + (size_t)b * A * D : NULL,
                            node_obs_out ? node_obs_out + (size_t)b * n * ND : NULL, NULL, NULL, NULL);
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(envs);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---------------------------------------------------------------------------
 * Batched driver for the CPU baseline (bench.py cpu_baseline leg): n_env
 * independent envs stepped with OpenMP; observations written to flat arrays.
 * ------------------------------------------------------------------------- */
gmo_env* gmo_batch_create(const gmo_config* c, int32_t n_env, uint32_t seed_base) {
    gmo_env* envs = (gmo_env*)malloc(sizeof(gmo_env) * (size_t)n_env);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < n_env; b++) gmo_env_init(&envs[b], c, seed_base + (uint32_t)b);
    return envs;
}

void gmo_batch_free(gmo_env* envs) { free(envs); }

void gmo_batch_run(gmo_env* envs, int32_t n_env, int32_t do_reset, const int32_t* act, float* reward, uint8_t* done,
                   float* obs, int64_t obs_stride, float* node_obs, int32_t* agent_node, int32_t* nbr) {
    int A = envs[0].cfg.n_data, n = envs[0].cfg.n_nodes;
    int D = gmo_obs_dim(n), ND = gmo_node_obs_dim(n);
#pragma omp parallel for schedule(static)
    for (int b = 0; b < n_env; b++) {
        gmo_env* e = &envs[b];
        if (do_reset) {
            gmo_env_reset(e);
        } else {
            gmo_info info;
            gmo_env_step(e, act + (size_t)b * A, reward + (size_t)b * A, done + (size_t)b * A, &info);
        }
        float tmp[GMO_MAXA * (6 * GMO_MAXN + 10)];
        gmo_env_observe(e, tmp, node_obs + (size_t)b * n * ND, NULL, NULL, NULL);
        for (int a = 0; a < A; a++) {
            memcpy(obs + ((size_t)b * A + a) * obs_stride, tmp + (size_t)a * D, sizeof(float) * D);
            agent_node[(size_t)b * A + a] = e->now[a];
        }
        for (int j = 0; j < n; j++)
            for (int k = 0; k < 3; k++) nbr[((size_t)b * n + j) * 3 + k] = e->topo.nbr[j][k];
    }
}

/* graph_marl_amd.h — C ABI of the MI355X-native graph-marl hot path.
 *
 * One handle = one batch of n_env independent routing environments resident in
 * HBM of one device. Every entry point takes plain device pointers, sizes and a
 * hipStream_t (passed as void*); nothing here allocates on the step path.
 * Return value: 0 on success, a negative gm_status otherwise; gm_last_error()
 * returns a message for the calling thread's last failure.
 *
 * Reference interfaces replaced (paths relative to the reference repo root):
 *   gm_env_create / gm_env_destroy   Routing.__init__ + Network.__init__   src/env/routing.py:55-109, src/env/network.py:47-98
 *   gm_env_reset                     Routing.reset (+ Network.reset)        src/env/routing.py:160-178, src/env/network.py:366-371
 *   gm_env_step                      Routing.step                           src/env/routing.py:360-520
 *   gm_env_observe                   _get_observation / get_node_observation / get_node_agent_matrix /
 *                                    _get_data_adjacency / get_node_aux     src/env/routing.py:187-358, 522-539
 *   gm_obs_from_gemm                 _get_observation rows rebuilt from the GEMM-ready copy  src/env/routing.py:269-315
 *   gm_env_topology                  get_nodes_adjacency (+ neighbour table) src/env/routing.py:184-185, src/env/network.py:385-389
 *   gm_env_final_info                Routing.get_final_info                 src/env/routing.py:541-546
 *   gm_build_seed_list               Network.build_seed_list                src/env/network.py:100-120
 *   gm_policy_egreedy                EpsilonGreedy.__call__ (draws + select) src/policy.py:20-64
 *   gm_env_policy_step               EpsilonGreedy.__call__ + Routing.step in one launch (src/main.py:701-703)
 *   gm_mp_aggregate(_bwd)            SimpleAggregation.forward              src/model.py:206-229
 *   gm_netmon_readout(_bwd)          NetMon._get_neighbor_h + output_to_network_obs src/model.py:582-631
 *   gm_lstm_pointwise(_bwd)          nn.LSTMCell gate math / LayerNorm-free part    src/model.py:379-382, 491, 543
 *   gm_linear_f32                    nn.Linear (+ leaky_relu of MLP)        src/model.py:13-42, 119-125
 *   gm_gemm_f32                      Linear / LSTMCell GEMMs with aggregate, readout and gate math fused
 *   gm_gemm_x3 / gm_gemm_pack_x3     the same GEMMs in split-f16 form (f16 MFMA, fp32 accumulate)
 *   gm_gemm_x3_head                  last DQN layer + Q head in one kernel
 *   gm_absmax_scale(_rows/_finish)   power-of-two operand scale for gm_gemm_x3 (input gradients)
 *   gm_gemm_x3_wgrad(2)              split-K weight-gradient GEMM over K-major operands (two B sources)
 *   gm_gemm_x3_dgrad / gm_lstm_cell_bwd / gm_qhead_bwd   backward of Linear+leaky_relu, LSTMCell and
 *                                    Q_Net.fc (torch autograd of the update, src/main.py:996)
 *   gm_agent_attention               AttModel attention core (DGN)          src/model.py:86-117
 *   gm_agent_comm                    CommNet communication step             src/model.py:780-787
 */
#ifndef GRAPH_MARL_AMD_H
#define GRAPH_MARL_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    GM_OK = 0,
    GM_ERR_INVALID_ARG = -1,
    GM_ERR_OOM = -2,
    GM_ERR_HIP = -3,
    GM_ERR_TOPOLOGY = -4, /* a provided topology seed is invalid / generator retry limit hit */
    GM_ERR_UNSUPPORTED = -5,
    GM_ERR_RANGE = -6 /* a split-f16 GEMM saw an operand outside the f16 range (gm_gemm_range_status) */
} gm_status;

/* topology modes: Network seed handling, src/env/network.py:215-272, 356-371 */
typedef enum {
    GM_TOPO_FIXED = 0,      /* --random-topology=0: one seed, no main-stream draw            */
    GM_TOPO_RANDOM = 1,     /* --random-topology=1 --num-topologies-train=0: fresh seed/reset */
    GM_TOPO_LIST = 2,       /* seed list, np.random.choice per reset                          */
    GM_TOPO_SEQUENTIAL = 3  /* seed list walked in order per env (evaluation over EVAL_SEEDS) */
} gm_topo_mode;

typedef struct {
    int32_t n_env;
    int32_t n_nodes;        /* --n-router, even, 4..128          */
    int32_t n_data;         /* --n-data (agents), <= 64          */
    int32_t env_var;        /* --env-var: 1 INDEPENDENT, 2 WITH_K_NEIGHBORS, 3 GLOBAL (routing.py:268-358) */
    int32_t congestion;     /* !--no-congestion                  */
    int32_t action_mask;    /* --action-mask                     */
    int32_t ttl;            /* --ttl (0 disables)                */
    int32_t topo_mode;      /* gm_topo_mode                      */
    int64_t topo_seed;      /* --topology-init-seed (FIXED)      */
    const int64_t* seed_list;  /* host, LIST / SEQUENTIAL        */
    int32_t n_seed_list;
    const int64_t* excluded;   /* host, seeds never used (EVAL_SEEDS); may be NULL */
    int32_t n_excluded;
    int32_t device;         /* HIP device ordinal                */
    int32_t k;              /* env_var 2: neighbour slots per observation, 0..8 (reference default 3) */
} gm_env_config;

/* Optional observation outputs (any pointer may be NULL). */
typedef struct {
    float* obs;             /* [n_env, A, obs_row_stride]; columns [0, obs_dim) written: 6N+10,
                               +5k (env_var 2), +N^2+N(4N+8) (env_var 3) — gm_env_dims     */
    int64_t obs_row_stride; /* floats between agent rows (>= obs_dim; obs_dim+512 with NetMon) */
    float* node_obs;        /* [n_env, N, 4N+8]                                           */
    int32_t* agent_node;    /* [n_env, A] node index of every agent (node-agent matrix)   */
    int8_t* agent_adj;      /* [n_env, A, A] agent adjacency                              */
    /* env_var 1 only: a GEMM-ready copy of each agent row without its two linearly dependent
     * columns, N-1 (= sum of the target one-hot - the other N-1 position one-hots) and 2N (edge
     * flag = sum of the next-hop one-hot): 6N+8 columns, column c = obs column c (c < N-1),
     * c+1 (c < 2N-1), c+2 (else). The DQN's first layer folds the two weight columns into the
     * others and runs with K = 6N+8 (640 with the readout at N = 20: whole 32-deep k tiles). */
    float* obs_gemm;        /* [n_env, A, obs_gemm_stride], 16-byte rows (nullable)        */
    int64_t obs_gemm_stride;
    /* obs NULL with obs_gemm set: the kernels write the GEMM-ready copy only (one copy of the
     * agent rows per step instead of two); gm_obs_from_gemm rebuilds obs rows from it. */
} gm_obs_buffers;

/* Per-env statistics of one step (src/env/routing.py:499-508), float64 [n_env, GM_INFO_FIELDS]. */
enum {
    GM_INFO_LOOPED = 0, GM_INFO_THROUGHPUT, GM_INFO_DROPPED, GM_INFO_BLOCKED,
    GM_INFO_N_DELAYS, GM_INFO_SUM_DELAYS, GM_INFO_N_ARRIVED, GM_INFO_SUM_DELAYS_ARRIVED,
    GM_INFO_SUM_SPR, GM_INFO_FIELDS
};

/* Eval-only statistics after the admission phase (src/env/routing.py:414-441, enabled by
 * set_eval_info), float64 [n_env, GM_EVAL_FIELDS]; the per-packet lists packet_sizes and
 * packet_distances are reported as sums over the A packets. */
enum {
    GM_EVAL_TOTAL_EDGE_LOAD = 0, GM_EVAL_OCCUPIED_EDGES, GM_EVAL_PACKETS_ON_EDGES, GM_EVAL_TOTAL_PACKET_SIZE,
    GM_EVAL_SUM_PACKET_DISTANCES, GM_EVAL_FIELDS
};

/* Optional per-packet step outputs for exact info lists (NULL to skip). */
typedef struct {
    int32_t* done_steps;    /* [n_env, A] agent steps of a packet that finished this step, else 0 */
    int32_t* done_opt;      /* [n_env, A] max(shortest path weight, 1) of that packet             */
    uint8_t* success;       /* [n_env, A] reached its target                                      */
    double* eval;           /* [n_env, GM_EVAL_FIELDS] eval-only statistics                       */
} gm_step_detail;

typedef struct gm_env gm_env;

const char* gm_last_error(void);
int gm_version(void);

int gm_env_create(const gm_env_config* cfg, const uint32_t* env_seeds /* host [n_env] */, gm_env** out);
int gm_env_destroy(gm_env* env);
int gm_env_dims(const gm_env* env, int32_t* n_env, int32_t* n_nodes, int32_t* n_data, int32_t* obs_dim,
                int32_t* node_obs_dim);

/* reset_mask: device uint8 [n_env] (NULL = every env). */
int gm_env_reset(gm_env* env, const uint8_t* reset_mask, const gm_obs_buffers* obs, void* stream);
/* actions: device int32 [n_env, A] in {0..3}; reward float32 [n_env, A]; done uint8 [n_env, A];
 * info float64 [n_env, GM_INFO_FIELDS] (nullable); detail nullable; obs nullable. */
int gm_env_step(gm_env* env, const int32_t* actions, float* reward, uint8_t* done, double* info,
                const gm_step_detail* detail, const gm_obs_buffers* obs, void* stream);
int gm_env_observe(gm_env* env, const gm_obs_buffers* obs, void* stream);
/* Agent observation rows (env_var 1: columns [0, 6N+10)) rebuilt from their GEMM-ready copies:
 * obs_gemm [rows, ld_gemm] (6N+8 columns, gm_obs_buffers.obs_gemm) -> obs [rows, ld_obs]. The
 * two dropped columns are restored exactly (column N-1 = sum of the target one-hot - the other
 * position one-hots; column 2N = sum of the next-hop one-hot), so the result equals what the env
 * kernels write into gm_obs_buffers.obs bit for bit. N even, 16-byte rows. */
int gm_obs_from_gemm(const float* obs_gemm, int64_t ld_gemm, int64_t rows, int32_t n_nodes, float* obs, int64_t ld_obs,
                     void* stream);
/* nbr: int32 [n_env, N, 3] neighbour ids ascending (= order of actions 1..3);
 * node_adj: int8 [n_env, N, N] (I + A); node_aux: float32 [n_env, N, N] APSP weights;
 * topo_seed: int64 [n_env]. Any may be NULL. */
int gm_env_topology(gm_env* env, int32_t* nbr, int8_t* node_adj, float* node_aux, int64_t* topo_seed,
                    void* stream);
/* ShortestPath heuristic (src/policy.py:90-139): actions int32 [n_env, A] = 1 + index (by
 * neighbour id) of the first hop of networkx's weighted shortest path now -> target
 * (Dijkstra with networkx's tie-breaking, src/env/network.py:279), 0 at the target. */
int gm_policy_shortest_path(gm_env* env, int32_t* actions, void* stream);
/* first-hop table int32 [n_env, N, N]: out[s][t] = next node on the s -> t path (t on the
 * diagonal) — network.shortest_paths[s][t][1] (src/env/network.py:279) */
int gm_env_first_hops(gm_env* env, int32_t* out, void* stream);
/* Switch the topology source between resets (the reference's evaluation sets
 * network.seeds = EVAL_SEEDS and sequential_topology_seeds = True, src/main.py:553-560,
 * 1049-1053). The sequential index restarts at 0 (network.py:87); with interleave, env b
 * starts at seed b and advances by n_env, so n_env envs walk the list like one env's
 * consecutive episodes. Synchronous. */
int gm_env_set_topology(gm_env* env, int32_t topo_mode, int64_t topo_seed, const int64_t* seed_list,
                        int32_t n_seed_list, int32_t interleave);
/* Sum and count of non-zero agent steps per env (get_final_info), float64 [n_env, 2]. */
int gm_env_final_info(gm_env* env, double* out, void* stream);

/* Network.build_seed_list (src/env/network.py:100-120) on the device: `count` unique
 * valid topology seeds from `init_seed` (EVAL_SEEDS = (20, 476, 1000)). out: host. */
int gm_build_seed_list(int32_t n_nodes, int64_t init_seed, int32_t count, const int64_t* excluded,
                       int32_t n_excluded, int32_t device, int64_t* out);

/* ε-greedy action selection: q float32 [n_env, A, 4]; epsilon as the reference's
 * float64; draws randint(4,size=A) then rand(A) from every env's stream. */
int gm_policy_egreedy(gm_env* env, const float* q, double epsilon, int32_t* actions, void* stream);
/* gm_policy_egreedy followed by gm_env_step as one kernel: the same draws in the same stream
 * order, so actions and every output are identical to the two calls; actions (device int32
 * [n_env, A]) receives the drawn actions. q must be 16-byte aligned. */
int gm_env_policy_step(gm_env* env, const float* q, double epsilon, int32_t* actions, float* reward, uint8_t* done,
                       double* info, const gm_step_detail* detail, const gm_obs_buffers* obs, void* stream);

/* Host-side state export/import for parity tests (synchronous). Arrays are host
 * pointers sized [n_env, ...]; any may be NULL. */
typedef struct {
    int32_t *now, *target, *edge, *time, *ttl, *start, *spw, *agent_steps; /* [n_env, A] */
    double* size;                                                          /* [n_env, A] */
    uint64_t* visited;                                                     /* [n_env, A, 2] */
    uint8_t* amask;                                                        /* [n_env, A, 4] */
    double* loads;                                                         /* [n_env, 3N/2] */
    int64_t* topo_seed;                                                    /* [n_env] */
    int32_t* topo_reps;                                                    /* [n_env] */
    int32_t *edge_a, *edge_b, *edge_len;                                   /* [n_env, 3N/2] */
    int32_t* nbr_edge;                                                     /* [n_env, N, 3] */
    int32_t* apsp;                                                         /* [n_env, N, N] */
    uint32_t* rng_key;   /* [n_env, 624] current MT block  */
    int32_t* rng_pos;    /* [n_env]                          */
    int32_t* seq_index;  /* [n_env] next position in a sequential topology-seed list
                            (Network.sequential_topology_index, src/env/network.py:356-364) */
} gm_env_state;
int gm_env_get_state(gm_env* env, gm_env_state* st);
/* Inverse of gm_env_get_state (synchronous): restores every non-NULL field (host arrays, same
 * layout); the neighbour table is rebuilt from nbr_edge + edge_a/edge_b, the numpy stream from
 * (rng_key, rng_pos) (both or neither). Observation buffers are left as they are: call
 * gm_env_observe. Replaces restoring a pickled Routing/Network (the reference has no state API;
 * its parity dumps are the numpy RandomState + object state, src/env/routing.py:30-178). */
int gm_env_set_state(gm_env* env, const gm_env_state* st);

/* ---- NetMon message passing (graphs of fixed max degree, ELL neighbour table) ----
 * h: float32 [G*N, H] rows; nbr: int32 [G, N, deg] neighbour ids (-1 = none).
 * out[n] = Σ over {n} ∪ nbr(n) in ascending node order (mode 0 = sum, 1 = mean). */
int gm_mp_aggregate(const float* h, const int32_t* nbr, int32_t n_graphs, int32_t n_nodes, int32_t deg,
                    int32_t hidden, int32_t mode, float* out, void* stream);
/* gm_mp_aggregate over strided rows (row strides ldh / ldo in floats): aggregates the h part of
 * [h | c] state rows in place of the GEMM's AGGREGATE A source. */
int gm_mp_aggregate_rows(const float* h, int64_t ldh, const int32_t* nbr, int32_t n_graphs, int32_t n_nodes,
                         int32_t deg, int32_t hidden, int32_t mode, float* out, int64_t ldo, void* stream);
/* LayerNorm-LSTM cell after its gate GEMMs (src/layernormlstm.py:24-42, NetMon rnn_type lnlstm):
 * g rows [m][ldg] hold [x W_ih^T | h W_hh^T] (8H floats, gate order i, f, g, o, no bias);
 * gates = LN(gi; ln_in_w, ln_in_b) + LN(gh; ln_hid_w, ln_hid_b) + bias, c1 = LN(sigma(f) c +
 * sigma(i) tanh(g); ln_cell_w, ln_cell_b), h1 = sigma(o) tanh(c1); LayerNorm eps as given
 * (torch default 1e-5). H <= 512; c, h1, c1 strided rows. */
int gm_lnlstm_pointwise(const float* g, int64_t ldg, const float* c, int64_t ldc, const float* ln_in_w,
                        const float* ln_in_b, const float* ln_hid_w, const float* ln_hid_b, const float* bias,
                        const float* ln_cell_w, const float* ln_cell_b, int32_t m, int32_t H, float eps, float* h1,
                        int64_t ldh, float* c1, int64_t ldc1, void* stream);
/* Training forms of the LayerNorm-LSTM cell (replace LayerNormLSTMCell.forward under autograd,
 * src/layernormlstm.py:24-42; the reference differentiates it with torch autograd). gm_lnlstm_fwd:
 * as gm_lnlstm_pointwise with the two gate GEMM outputs as separate strided row sets gi, gh
 * ([m][4H] each) and the row statistics stats[m][8] = (mean, 1/std) of gi, gh and the cell
 * pre-norm saved for gm_lnlstm_bwd. gm_lnlstm_bwd: dh1 / dc1 (either nullable) -> d gi, d gh
 * ([m][4H] strided), d c ([m][H]) and per-wave parameter-gradient partials part[ceil(m /
 * rows_per_wave)][14H] = [d ln_in_w (4H) | d ln_hid_w (4H) | d bias (4H; equal to d ln_in_b and
 * d ln_hid_b) | d ln_cell_w (H) | d ln_cell_b (H)] (the caller sums the rows). */
int gm_lnlstm_fwd(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* c, int64_t ldc,
                  const float* ln_in_w, const float* ln_in_b, const float* ln_hid_w, const float* ln_hid_b,
                  const float* bias, const float* ln_cell_w, const float* ln_cell_b, int32_t m, int32_t H, float eps,
                  float* h1, int64_t ldh, float* c1, int64_t ldc1, float* stats, void* stream);
int gm_lnlstm_bwd(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* c, int64_t ldc,
                  const float* ln_in_w, const float* ln_in_b, const float* ln_hid_w, const float* ln_hid_b,
                  const float* bias, const float* ln_cell_w, const float* ln_cell_b, const float* stats,
                  const float* dh1, int64_t lddh, const float* dc1, int64_t lddc, int32_t m, int32_t H,
                  int32_t rows_per_wave, float* dgi, int64_t lddgi, float* dgh, int64_t lddgh, float* dc,
                  int64_t lddco, float* part, void* stream);
/* GRU cell gate math (torch.nn.GRUCell, used by NetMon rnn_type gru, src/model.py:387-393) after its
 * two GEMMs gi = x W_ih^T + b_ih, gh = h W_hh^T + b_hh ([m][3H] strided, gates r, z, n):
 * h1 = (1 - z) n + z h. gm_gru_bwd: dh1 -> d gi, d gh ([m][3H]) and the direct d h ([m][H]). */
int gm_gru_pointwise(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* h, int64_t ldh,
                     int32_t m, int32_t H, float* h1, int64_t ldh1, void* stream);
int gm_gru_bwd(const float* gi, int64_t ldgi, const float* gh, int64_t ldgh, const float* h, int64_t ldh,
               const float* dh1, int64_t lddh1, int32_t m, int32_t H, float* dgi, int64_t lddgi, float* dgh,
               int64_t lddgh, float* dh, int64_t lddh, void* stream);
/* Backward of a Linear followed by leaky_relu (MLP layers, src/model.py:13-42): g = dY where
 * Y >= 0 else slope * dY ([rows][cols] contiguous), and per-block column sums of g for the bias
 * gradient: part[ceil(rows / rows_per_block)][cols] (the caller sums the blocks); g_scale
 * (nullable) receives the power-of-two scale of g (as gm_absmax_scale, without a second pass). */
int gm_leaky_bwd(const float* dy, const float* y, int64_t rows, int32_t cols, float slope, float* g, float* part,
                 int32_t rows_per_block, float* g_scale, void* stream);
/* The same for any GM_ACT_* layer activation (derivative from the output y: relu y > 0, elu
 * y > 0 ? 1 : y + 1, tanh 1 - y^2, sigmoid y (1 - y); replaces torch autograd of the reference's
 * activation_fn, src/model.py:13-42). */
int gm_act_bwd(const float* dy, const float* y, int64_t rows, int32_t cols, int32_t act, float* g, float* part,
               int32_t rows_per_block, float* g_scale, void* stream);
/* Activations whose derivative needs the pre-activation z (GM_ACT_GELU.., torch autograd of the
 * reference's activation_fn, src/model.py:13-42): y = act(z) elementwise ([rows][cols] contiguous),
 * and the backward g = dY * act'(z) with the per-block column sums and g_scale of gm_act_bwd. Both take
 * every GM_ACT_* code. */
int gm_act_fwd(const float* z, int64_t rows, int32_t cols, int32_t act, float* y, void* stream);
int gm_act_bwd_z(const float* dy, const float* z, int64_t rows, int32_t cols, int32_t act, float* g, float* part,
                 int32_t rows_per_block, float* g_scale, void* stream);
/* SL regression loss at every unroll step (src/sl.py:396-400: mse_loss(pred_all, targets_all) after each
 * of the L steps; replaces torch's mse_loss and its autograd): pred [L][n] contiguous, tgt [n] (the same
 * target at every step), n % 4 == 0, 16-byte bases. gm_step_mse writes per-block partial sums of squared
 * differences, part [L][gm_step_mse_blocks(n)] (the caller sums each row in order and divides by n);
 * gm_step_mse_bwd writes grad[l][i] = (pred[l][i] - tgt[i]) * (g[l] * two_over_n) with g the L upstream
 * gradients of the per-step losses and two_over_n = 2 / n rounded to float. */
int32_t gm_step_mse_blocks(int64_t n);
int gm_step_mse(const float* pred, const float* tgt, int64_t n, int32_t L, float* part, void* stream);
int gm_step_mse_bwd(const float* pred, const float* tgt, int64_t n, int32_t L, const float* g, float two_over_n,
                    float* grad, void* stream);
/* Backward of gm_mp_aggregate for symmetric adjacency: dh[j] = Σ_{n ∈ {j} ∪ nbr(j)} dout[n] / cnt(n). */
int gm_mp_aggregate_bwd(const float* dout, const int32_t* nbr, int32_t n_graphs, int32_t n_nodes, int32_t deg,
                        int32_t hidden, int32_t mode, float* dh, void* stream);
/* Readout (NetMon.forward with output_neighbor_hidden) fused with the agent gather:
 * row r of graph g maps to node v = agent_node[g*R + r] (or v = r when agent_node is NULL, R = N);
 * out[g*R + r] = [h_final[v], h_prev[nbr(v,0)], ..., h_prev[nbr(v,deg-1)]] (zeros for -1),
 * written at out + (g*R + r) * out_stride (floats). */
int gm_netmon_readout(const float* h_final, const float* h_prev, const int32_t* nbr, const int32_t* agent_node,
                      int32_t n_graphs, int32_t n_nodes, int32_t n_rows, int32_t deg, int32_t hidden, float* out,
                      int64_t out_stride, void* stream);
/* Its backward: dh_final[v] / dh_prev[u] = the sums of the dout segments that read them (either output
 * nullable). Without an agent map (agent_node NULL, n_rows = n_nodes: every node read out, config 5) the
 * neighbour table must be symmetric (u in nbr(v) <=> v in nbr(u): the routing graphs are), and dh_prev[u] is
 * gathered from u's neighbours' rows (ascending, the same fp32 sums as the general form). */
int gm_netmon_readout_bwd(const float* dout, int64_t dout_stride, const int32_t* nbr, const int32_t* agent_node,
                          int32_t n_graphs, int32_t n_nodes, int32_t n_rows, int32_t deg, int32_t hidden,
                          float* dh_final, float* dh_prev, void* stream);
/* LSTM gate math: gates [M, 4H] pre-activations (i,f,g,o, biases included), c [M, H]
 * -> h_new, c_new [M, H]; saves sigmoid/tanh activations in act [M, 4H] if non-NULL. */
int gm_lstm_pointwise(const float* gates, const float* c, int32_t m, int32_t hidden, float* h_new, float* c_new,
                      float* act, void* stream);
/* Backward: given dh_new, dc_new (nullable = 0), act, c, c_new -> dgates [M,4H], dc [M,H];
 * dgates_scale (nullable) receives the power-of-two scale of dgates (as gm_absmax_scale). */
int gm_lstm_pointwise_bwd(const float* dh_new, const float* dc_new, const float* act, const float* c,
                          const float* c_new, int32_t m, int32_t hidden, float* dgates, float* dc,
                          float* dgates_scale, void* stream);
/* LSTM cell backward of the sequence-batched training path (nn.LSTMCell, src/model.py:379-382,
 * 491, 543, backward of torch autograd): per row r and unit u, with gate activations act (i, f,
 * g, o), cell input c and output c' = c_out:
 *   dh = dh0 + dh1 + sum_{n in {r} U nbr(r)} dm[n] s(n) + (ext_mask[r / rows_per_sample] ? 0 : dh_ext)
 *   dc' = dc + (ext_mask[...] ? 0 : dc_ext)
 * (every source nullable; dm = the input gradient of the aggregate input of the next cell,
 * s(n) = 1 or 1 / |{n} U nbr(n)| for mean); writes dgates (i, f, g, o pre-activation gradients),
 * dc_out = dc'_total * f (nullable), per-block column sums of dgates to bias_part
 * [ceil(m / rows_per_block)][4H] (nullable), max |dgates| to dg_scale as a power-of-two scale
 * (gm_absmax_scale semantics, nullable) and as float bits into dg_max (nullable, accumulated by
 * atomicMax). H <= 256, 256 % H == 0 or H % 64 == 0 with H <= 1024. */
typedef struct {
    const float* act; int64_t ld_act;
    const float* c_in; int64_t ld_cin;
    const float* c_out; int64_t ld_cout;
    const float* dh0; int64_t ld_dh0;
    const float* dh1; int64_t ld_dh1;
    const float* dm; int64_t ld_dm;
    const int32_t* nbr; int32_t n_nodes, deg, mean;
    const float* dh_ext; int64_t ld_ext;
    const float* dc_ext; int64_t ld_dcext;
    const uint8_t* ext_mask; int32_t rows_per_sample;
    const float* dc; int64_t ld_dc;
    int32_t m, hidden;
    float* dgates; int64_t ld_dg;
    float* dc_out; int64_t ld_dco;
    float* bias_part; int32_t rows_per_block;
    float* dg_scale;
    float* dg_max;
} gm_lstm_bwd_args;
int gm_lstm_cell_bwd(const gm_lstm_bwd_args* a, void* stream);
/* Q head + last hidden layer backward (Q_Net.fc after a leaky_relu MLP layer, src/model.py:119-125,
 * 187-203): g[r][c] = (sum_a dq[r][a] wq[a][c]) * (act && y[r][c] <= 0 ? 0.01 : 1) for the layer
 * output y; per block of rows_per_block rows: part_b[blk][c] = sum g (the layer's bias gradient),
 * part_wq[blk][a][c] = sum dq[r][a] y[r][c] (the head's weight gradient), part_bq[blk][a] =
 * sum dq[r][a]; g_scale (nullable): power-of-two scale of g (gm_absmax_scale semantics).
 * nq <= 4, cols <= 1024. */
int gm_qhead_bwd(const float* dq, int64_t ldq, int32_t nq, const float* wq, int64_t ldwq, const float* y,
                 int64_t ldy, int64_t rows, int32_t cols, int32_t act, float* g, int64_t ldg, float* part_b,
                 float* part_wq, float* part_bq, int32_t rows_per_block, float* g_scale, void* stream);
/* gm_netmon_readout with strided h rows (h_final [.][ldf], h_prev [.][ldp]; e.g. the [h | c]
 * state rows of the LSTM, ld = 2H). */
int gm_netmon_readout_ld(const float* h_final, int64_t ldf, const float* h_prev, int64_t ldp, const int32_t* nbr,
                         const int32_t* agent_node, int32_t n_graphs, int32_t n_nodes, int32_t n_rows, int32_t deg,
                         int32_t hidden, float* out, int64_t out_stride, void* stream);
/* Fused f32 MFMA linear layer: y[M,N] = act(x[M,K] @ w[N,K]^T + b[N]); row strides ldx, ldw
 * (multiples of 4 floats, 16-byte aligned bases), ldy; K may be ragged; b nullable;
 * act 0 = none, 1 = leaky_relu(0.01). */
int gm_linear_f32(const float* x, int64_t ldx, const float* w, int64_t ldw, const float* b, int32_t m, int32_t n,
                  int32_t k, int32_t act, float* y, int64_t ldy, void* stream);

/* ---- General fused GEMM: y = epilogue(A @ W^T + b), A = [src0 | src1] along K ----
 * Replaces the reference's Linear layers of MLP/DQN (src/model.py:13-42, 187-203) and the
 * LSTMCell gate GEMM (src/model.py:379-382) with the aggregate (206-229) and the readout +
 * agent gather (582-631) folded into the A-operand load. */
enum { GM_A_DENSE = 0, GM_A_AGGREGATE = 1, GM_A_READOUT = 2, GM_A_ROUTING_ENC = 3 };
enum { GM_EPI_BIAS = 0, GM_EPI_BIAS_LEAKY = 1, GM_EPI_LSTM = 2, GM_EPI_GRU = 3, GM_EPI_BIAS_RELU = 4,
       GM_EPI_BIAS_ELU = 5, GM_EPI_BIAS_TANH = 6, GM_EPI_BIAS_SIGMOID = 7, GM_EPI_BIAS_ACT = 64 };
/* Layer activations (--activation-function = any elementwise torch.nn.functional name with its
 * defaults, src/main.py:194-197, 440-441; MLP / AttModel, src/model.py:13-42, 86-117). Codes
 * 1..GM_ACT_SOFTPLUS have a derivative that follows from the layer output y (the training backward
 * keeps y); codes GM_ACT_GELU.. need the pre-activation z (the training forward keeps z and applies
 * the activation with gm_act_fwd). GM_EPI_BIAS_<ACT> (4..7) or GM_EPI_BIAS_ACT + act (any code) =
 * bias + activation epilogue; act arguments take GM_ACT_*. */
enum { GM_ACT_NONE = 0, GM_ACT_LEAKY_RELU = 1, GM_ACT_RELU = 2, GM_ACT_ELU = 3, GM_ACT_TANH = 4, GM_ACT_SIGMOID = 5,
       GM_ACT_RELU6 = 6, GM_ACT_HARDTANH = 7, GM_ACT_HARDSIGMOID = 8, GM_ACT_SELU = 9, GM_ACT_CELU = 10,
       GM_ACT_SOFTSIGN = 11, GM_ACT_LOGSIGMOID = 12, GM_ACT_SOFTPLUS = 13, GM_ACT_GELU = 14, GM_ACT_SILU = 15,
       GM_ACT_MISH = 16, GM_ACT_HARDSWISH = 17, GM_ACT_TANHSHRINK = 18, GM_ACT_LAST = 18 };
typedef struct {
    int32_t mode;              /* GM_A_*                                                           */
    const float* p0;           /* DENSE: rows; AGGREGATE: node rows h; READOUT: h_final node rows  */
    const float* p1;           /* READOUT: h_prev node rows (the last pre-aggregation h)           */
    int64_t ld0, ld1;          /* row strides in floats (multiples of 4)                           */
    const int32_t* nbr;        /* AGGREGATE / READOUT: [G][n_nodes][deg] ascending, -1 = none      */
    const int32_t* agent_node; /* READOUT: [G * rows_per_graph] node of every row                  */
    int32_t n_nodes, deg, mean, rows_per_graph;
    int32_t k;                 /* columns this source contributes (READOUT: (deg + 1) * hidden)    */
    int32_t hidden;            /* READOUT: H (multiple of 32)                                      */
    const float* scale;        /* gm_gemm_x3, DENSE src0 without src1 (nullable): device power of  */
                               /* two s from gm_absmax_scale; A is split as s*A, the result / s    */
    uint32_t* amax;            /* gm_gemm_x3, src0 (nullable): max |A| over [src0 | src1] published */
                               /* as float bits by atomicMax (zero it first; gm_absmax_finish)      */
    const float* bias0;        /* ROUTING_ENC (nullable): bias of the folded encoder layer          */
    int32_t act0;              /* ROUTING_ENC: its activation (GM_ACT_*)                            */
} gm_a_src;
/* GM_A_ROUTING_ENC (gm_gemm_x3 only, no src1): A = act0(W0 x + b0), the NetMon encoder's first layer
 * (src/model.py:13-42, 489) on routing node observations x (src/env/routing.py:187-235: [onehot(n) | cnt |
 * load | 3 x (onehot(nbr_k) | len_k | load_k)], 4N + 8 columns) computed inside the GEMM's A-tile load from
 * the 12 nonzero columns, so the m x k layer output never reaches HBM: p0 = x rows ([G * n_nodes][ld0]),
 * p1 = W0^T ([4N + 8][ld1], ld1 >= k), nbr = [G][n_nodes][3] (deg = 3, every entry a node id in [0, N): the
 * routing graphs are 3-regular; -1 entries are NOT masked here, unlike READOUT), n_nodes = N with 4N + 8 <= 208 (N <= 50),
 * k = the layer's width (multiple of 32), bias0 / act0. Runs on v_mfma_f32_16x16x32_f16 (whatever
 * gm_gemm_set_mfma selects for the other GEMMs) and needs a bias epilogue; other cases return
 * GM_ERR_UNSUPPORTED (run gm_routing_node_encoder and a DENSE source instead). */
/* src1 (nullable) must be DENSE and src0->k a multiple of 32. W: [n][ldw] (ldw >= K, zero
 * padded to a multiple of 4). GM_EPI_LSTM: W rows packed so that rows [128t, 128t+128) are
 * gates i,f,g,o (32 rows each) of hidden units [32t, 32t+32); n = 4H; writes h' to y, c' to y2,
 * reads c from c_in, optional activations [M][4H] (original gate order) to act_out.
 * GM_EPI_GRU (torch.nn.GRUCell, reference NetMon rnn_type gru, src/model.py:387-389): A = [x | h],
 * n = 4H with rows [128t, 128t+128) = tiles r, z, n_x, n_h of hidden units [32t, 32t+32) where
 * r, z rows are [W_ih | W_hh], n_x rows [W_in | 0], n_h rows [0 | W_hn] (biases b_ir + b_hr,
 * b_iz + b_hz, b_in, b_hn); c_in = h; y = h' = (1 - z) n + z h with n = tanh(n_x + r n_h); y2 unused. */
int gm_gemm_f32(const gm_a_src* src0, const gm_a_src* src1, const float* w, int64_t ldw, const float* b, int32_t m,
                int32_t n, int32_t epilogue, float* y, int64_t ldy, float* y2, int64_t ldy2, const float* c_in,
                int64_t ldc, float* act_out, void* stream);
/* Same GEMM in split-f16 form (the rollout's default): every operand a = a_hi + a_lo with
 * f16 pieces (22 significant bits), a·w = a_hi·w_hi + a_hi·w_lo + a_lo·w_hi on
 * v_mfma_f32_32x32x16_f16 with fp32 accumulation — 5.3x fewer MFMA cycles than the f32
 * form; error vs fp64 the order of an fp32 GEMM's (tests/test_fused_gpu.py). A stays fp32
 * in HBM (split while staged to LDS); wp = weights packed by gm_gemm_pack_x3 for the same
 * (n, K = src0->k + src1->k), wscale_inv its device scalar. Arguments otherwise as
 * gm_gemm_f32. Range: an A element whose split leaves the f16 range (|a| >= 65520, or a low
 * piece (a - a_hi) * 2^12 >= 65520, possible from |a| >= 2^15) turns its row's accumulators
 * inf/NaN; the kernel then sets a host-mapped status word, and every later gm_gemm_x3 /
 * gm_gemm_x3_head call fails with GM_ERR_RANGE until gm_gemm_range_status clears it. */
int gm_gemm_x3(const gm_a_src* src0, const gm_a_src* src1, const void* wp, const float* wscale_inv, const float* b,
               int32_t m, int32_t n, int32_t epilogue, float* y, int64_t ldy, float* y2, int64_t ldy2,
               const float* c_in, int64_t ldc, float* act_out, void* stream);
/* (gm_gemm_x3, GM_EPI_BIAS / GM_EPI_BIAS_LEAKY: act_out, when given, receives the sign bits of y
 * (bit c % 32 of uint32 word [row][c / 32] set when y > 0; ldc = words per row >= ceil(n / 32)):
 * the leaky_relu derivative the training backward's gm_gemm_x3_dgrad reads, 1/32 of y's bytes.) */
/* Status of the split-f16 range guard (no stream synchronisation: the word is host memory the
 * kernels write): *status = 1 when a gm_gemm_x3 / gm_gemm_x3_head launch that has finished
 * produced a non-finite accumulator since the last clear; clear != 0 resets it. Callers check
 * it at their synchronisation points (episode ends, after an update). */
int gm_gemm_range_status(int32_t* status, int32_t clear);
/* Last DQN encoder layer + Q head in one kernel (split-f16 form for the layer, fp32 head):
 * q[m][nq] = Wq · act(src0 · W^T + b) + bq, act 0 none / 1 leaky_relu(0.01); the hidden
 * activation stays in registers (also written to y when y != NULL). src0 DENSE, n <= 256,
 * nq <= 4, wq [nq][ldwq] fp32; src0->amax (nullable) receives max |src0| (training forward).
 * Replaces encoder.linear_layers[-1] + Q_Net.fc of the reference DQN (src/model.py:119-125,
 * 187-203). */
int gm_gemm_x3_head(const gm_a_src* src0, const void* wp, const float* wscale_inv, const float* b, int32_t m,
                    int32_t n, int32_t act, const float* wq, int64_t ldwq, const float* bq, int32_t nq, float* q,
                    int64_t ldq, float* y, int64_t ldy, void* stream);
/* The rollout's NetMon encoder (src/model.py:13-42 MLP, 489) in ONE launch: layer 1 computed in layer 2's
 * A-tile load from the routing node observations (a0: GM_A_ROUTING_ENC), layer 2 (n2 = 256) kept on chip
 * per 128-row block as split-f16 LDS images, layer 3 (n3 = 128) from them; y [m][ldy] = act3(act2(A W2^T +
 * b2) W3^T + b3). w2p / w2sinv, w3p / w3sinv: gm_gemm_pack_x3 of W2 [256][k] and W3 [128][256]. Neither the
 * m x k layer-1 nor the m x 256 layer-2 activation is written. */
int gm_encoder_x3(const gm_a_src* a0, const void* w2p, const float* w2sinv, const float* b2, int32_t act2,
                  const void* w3p, const float* w3sinv, const float* b3, int32_t act3, int32_t m, int32_t n2, int32_t n3,
                  float* y, int64_t ldy, void* stream);
/* Input-gradient GEMM of a layer whose input went through leaky_relu (the reference MLP's
 * F.leaky_relu, src/model.py:13-42, backward of torch autograd, src/main.py:996): D = src0 . W^T
 * in split-f16 form over wp = gm_gemm_pack_x3 of W^T ([n][K], K = src0->k; src0 DENSE, its
 * power-of-two scale in src0->scale); columns < split: g = D * (input > 0 ? 1 : 0.01), the layer
 * input's sign given as bits (mask_bits [m][ldm] uint32 words: bit c % 32 of word c / 32 set when
 * input[c] > 0, as the forward epilogues write them; nullable = no derivative; ldm 0: one row for
 * all) to y [m][ldy], per-128-row-tile column
 * sums to part [ceil(m / 128)][split] (nullable; the bias gradient of the previous layer) and
 * max |g| as float bits to gmax (nullable, zeroed by the caller; gm_absmax_finish); columns >= split
 * unchanged to y2 [m][ldy2] (e.g. the LSTM [x | h] input gradient split into its parts). */
int gm_gemm_x3_dgrad(const gm_a_src* src0, const void* wp, const float* wscale_inv, int32_t m, int32_t n,
                     int32_t split, const uint32_t* mask_bits, int64_t ldm, float* y, int64_t ldy, float* y2,
                     int64_t ldy2, float* part, float* gmax, void* stream);
/* Weight-gradient GEMM of the training path: C_z = A_z^T B_z for k-splits z of kchunk rows
 * (K = batch rows): A = dY [k][lda], B = X [k][ldb], both K-major fp32, scaled by the device
 * powers of two sa, sb (gm_absmax_scale) and split into f16 pieces on the way into LDS;
 * partial C_z [m][ldc] at c + z*m*ldc (the caller sums the ceil(k / kchunk) partials). m, n,
 * lda, ldb multiples of 4, 16-byte bases, kchunk a multiple of 16. Replaces the weight
 * gradients of the reference's Linear / LSTMCell layers (torch autograd, src/main.py:840-1026). */
int gm_gemm_x3_wgrad(const float* a, int64_t lda, const float* b, int64_t ldb, int32_t m, int32_t n, int32_t k,
                     int32_t kchunk, const float* sa, const float* sb, float* c, int64_t ldc, void* stream);
/* One K-major B source of gm_gemm_x3_wgrad2: n columns of p (row stride ld floats, 16-byte base), operand scale
 * (device power of two, as sb); batch row r of a reads source row (period ? r % period : r) + shift, and zeros
 * where that row lies outside [0, rows) (period / shift: multiples of kchunk). E.g. the config-5 obs cell, whose
 * input x = E [M][H] is the same at every one of the L steps: period = M; its h input of step t is step t-1's
 * state [(L-1) M rows]: shift = -M (zero at t = 0). */
typedef struct {
    const float* p;
    int64_t ld;
    const float* scale;
    int64_t period, shift, rows;
} gm_wgrad_src;
/* The weight gradients of two B sources that share the gradient operand a, in ONE launch: c = a^T [b1 | b2]
 * (n1 columns of b1, n2 of b2; b2 nullable), split-K partials [k / kchunk][m][ldc >= n1 + n2]; each k chunk of a
 * is fetched once into the XCD's L2 for both (the LSTM cell's W_ih / W_hh, the DQN's first layer over [readout |
 * env obs]). n1 % 128 == 0 when b2 is given. */
int gm_gemm_x3_wgrad2(const float* a, int64_t lda, const gm_wgrad_src* b1, int32_t n1, const gm_wgrad_src* b2,
                      int32_t n2, int32_t m, int32_t k, int32_t kchunk, const float* sa, float* c, int64_t ldc,
                      void* stream);
/* s = 2^(14 - e) with max|x| in [2^(e-1), 2^e) (1 when x is all zero): the power-of-two scale
 * that brings a gm_gemm_x3 A operand of small magnitude (e.g. gradients) into the range where
 * both f16 pieces of the split are normal. x: n floats; scale: one device float. */
int gm_absmax_scale(const float* x, int64_t n, float* scale, void* stream);
/* The same scale for a [rows][cols] block with row stride ld (floats). */
int gm_absmax_scale_rows(const float* x, int64_t rows, int32_t cols, int64_t ld, float* scale, void* stream);
/* The same scale from a max already published by a producer (gm_gemm_x3's src0 amax,
 * gm_leaky_bwd, gm_lstm_pointwise_bwd): *scale holds max|x| as float bits on entry, the scale
 * on exit. */
int gm_absmax_finish(float* scale, void* stream);
/* Packed size in bytes of an [n][k] weight for gm_gemm_x3: n * ceil(k/32)*2 blocks * 64 B. */
int64_t gm_gemm_pack_x3_bytes(int32_t n, int32_t k);
/* Split W [n][ldw] (first k columns) into wp (16-byte aligned, gm_gemm_pack_x3_bytes):
 * per row and 16-deep k block, 16 f16 hi then 16 f16 lo of S*W, zero past k, with S = a
 * power of two that puts S*max|W| in [2^14, 2^15); writes 1/S to *wscale_inv (device).
 * Stream-ordered, no host sync. */
int gm_gemm_pack_x3(const float* w, int64_t ldw, int32_t n, int32_t k, void* wp, float* wscale_inv, void* stream);
/* First NetMon encoder layer on routing node observations (src/model.py:272-276 applied
 * to src/env/routing.py:187-235): y = act(W x + b) from the 12 nonzero entries of each node
 * row (own one-hot, packet count and load, per neighbour one-hot, edge length, edge load)
 * instead of the dense K = 4N+8 product. x: node obs rows [G*N][ldx]; nbr int32 [G][N][3]
 * ascending; wt = W^T [4N+8][n] row-major (16-byte aligned); b [n] or NULL; y [G*N][ldy].
 * n % 64 == 0; act 0 none, 1 leaky_relu(0.01). */
int gm_routing_node_encoder(const float* x, int64_t ldx, const int32_t* nbr, int32_t G, int32_t N,
                            const float* wt, const float* b, int32_t n, int32_t act, float* y, int64_t ldy,
                            void* stream);
/* The same, also writing the sign bits of y (as gm_gemm_x3's act_out; ldsb words per row). */
int gm_routing_node_encoder_bits(const float* x, int64_t ldx, const int32_t* nbr, int32_t G, int32_t N,
                                 const float* wt, const float* b, int32_t n, int32_t act, float* y, int64_t ldy,
                                 uint32_t* sbits, int64_t ldsb, void* stream);
/* ---- Agent models (DGN, CommNet): per-env A x A agent communication ----
 * gm_agent_attention (AttModel.forward, src/model.py:86-117): for every env b, agent i and
 * head h: w_ij = <q_i, k_j> / sqrt(dk); p = softmax_j(adj_ij ? w_ij : -1e9); out_i =
 * sum_j p_ij v_j + v_i. q, k, v: rows [B*A][ld] (head h at columns [h*d, (h+1)*d)), already
 * activated; adj int8 [B][A][A]; out rows [B*A][ldo] (heads concatenated); att_weights
 * (nullable) [B][heads][A][A] receives w (unmasked, like the reference). A <= 64, dk, dv <= 64. */
int gm_agent_attention(const float* q, const float* k, const float* v, int64_t ld, const int8_t* adj, int32_t B,
                       int32_t A, int32_t heads, int32_t dk, int32_t dv, float* out, int64_t ldo,
                       float* att_weights, void* stream);
/* gm_agent_comm (CommNet.forward, src/model.py:780-787): out_i = h_i + sum_{j != i, adj_ij}
 * h_j / max(count, 1) per env; h, out rows [B*A][ldh / ldo] (out must not alias h). */
int gm_agent_comm(const float* h, int64_t ldh, const int8_t* adj, int32_t B, int32_t A, int32_t H, float* out,
                  int64_t ldo, void* stream);

/* Build provenance: "src=<16 hex digits of the SHA-256 of the csrc sources and headers> arch=<gfx> hipcc=<version>",
 * fixed when the library is linked (tests/test_capi.py checks it against the tree; bench.py reports it). */
const char* gm_build_info(void);

/* Process-wide kernel-form switches for A/B timing live in graph_marl_amd_tuning.h. */
#include "graph_marl_amd_tuning.h"

/* ---------------------------------------------------------------------------
 * SimpleEnvironment (src/env/simple_environment.py:45-334; BASELINE config 1):
 * 3 routers on a line, 1 packet at the middle router, actions {0, 1}, reward = score
 * (-1/+1) of the router reached, done every step. Batched over n_env envs, each with
 * its own numpy-legacy stream (seeds[env]); reset draws exactly the reference's
 * sequence (_build_network 123-209), gm_simple_policy_egreedy draws EpsilonGreedy's
 * randint(2, size=1) + rand(1) (src/policy.py:44-50) from the same stream.
 * ------------------------------------------------------------------------- */
typedef struct gm_simple_env gm_simple_env;
typedef struct {
    float* obs;              /* [n_env][1][obs_row_stride]: [now] (+ adjacency 9 + scores 3 if env_var != 1) */
    int64_t obs_row_stride;
    float* node_obs;         /* [n_env][3][1] router scores (get_node_observation) */
    int8_t* node_adj;        /* [n_env][3][3] I + A (get_nodes_adjacency) */
    int32_t* nbr;            /* [n_env][3][2] neighbour ids ascending, -1 padded */
    int32_t* agent_node;     /* [n_env][1] router of the packet (get_node_agent_matrix) */
} gm_simple_obs;
typedef struct { /* host buffers, any may be NULL */
    int32_t* score;          /* [n_env][3] */
    int32_t* router_edge;    /* [n_env][3][2] Router.edge lists (-1 = none) */
    int32_t* edge_end;       /* [n_env][2][2] Edge (start, end) */
    int32_t* start;          /* [n_env] */
    int32_t* now;            /* [n_env] */
} gm_simple_state;
int gm_simple_create(int32_t n_env, int32_t env_var, int32_t random_topology, const uint32_t* seeds_host,
                     int32_t device, gm_simple_env** out);
int gm_simple_destroy(gm_simple_env* env);
/* SimpleEnvironment.reset (simple_environment.py:211-213); reset_mask (device u8 [n_env]) or NULL = all */
int gm_simple_reset(gm_simple_env* env, const uint8_t* reset_mask, const gm_simple_obs* obs, void* stream);
/* SimpleEnvironment.step (simple_environment.py:283-315): actions int32 [n_env] in {0, 1} */
int gm_simple_step(gm_simple_env* env, const int32_t* actions, float* reward, uint8_t* done,
                   const gm_simple_obs* obs, void* stream);
int gm_simple_observe(gm_simple_env* env, const gm_simple_obs* obs, void* stream);
int gm_simple_policy_egreedy(gm_simple_env* env, const float* q, double epsilon, int32_t* actions, void* stream);
/* synchronous; fails with GM_ERR_INVALID_ARG if an invalid action was stepped since the last call */
int gm_simple_get_state(gm_simple_env* env, gm_simple_state* st);

/* ---- Replay sampling stream (reference src/replaybuffer.py:101-130: np.random.default_rng(seed)
 * .choice(n, size, replace=True)) ----
 * numpy Generator state: PCG64 128-bit state and increment plus the buffered high half of the
 * last 64-bit output (has_uint32 / uinteger), exactly numpy's bit_generator.state. */
typedef struct gm_pcg64 {
    uint64_t state_hi, state_lo, inc_hi, inc_lo;
    uint32_t has_uint32, uinteger;
} gm_pcg64;
/* Host: numpy.random.default_rng(seed)'s initial state (SeedSequence(seed).generate_state(4,
 * uint64), PCG64 srandom) for 0 <= seed < 2^64. */
int gm_pcg64_seed(uint64_t seed, gm_pcg64* out);
/* Device: out[0..count) = Generator.choice(n, count, replace=True) (= integers(0, n, int64):
 * Lemire's bounded 32-bit draws with numpy's rejection rule) continuing the stream in `state`
 * (device memory, advanced in place, stream-ordered). 1 <= n <= 2^32 - 1. */
int gm_pcg64_choice(gm_pcg64* state, int64_t n, int64_t count, int64_t* out, void* stream);
/* Device: gather of sampled ring records (replaybuffer.get_sequences; the reference copies the sampled
 * rows of its host arrays, src/replaybuffer.py:103-130): dst + i * bytes <- src + slot[i] * ld_slot +
 * env[i % n_env_idx] * ld_env, `bytes` bytes, for i < n. Strides in bytes; records, strides and bases
 * 16-byte aligned; n * bytes / 16 < 2^31. */
int gm_gather_records(const void* src, int64_t ld_slot, int64_t ld_env, const int64_t* slot, const int64_t* env,
                      int32_t n_env_idx, int64_t n, int64_t bytes, void* dst, void* stream);

#ifdef __cplusplus
}
#endif
#endif

// rl_kparams.h — kernel parameter block and lane-record packing shared by the
// host runtime (rl_host.cpp) and the gfx950 kernels (rl_train_*.hip).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#include "rl.h"

#ifndef RLAMD_EXP
#define RLAMD_EXP 0
#endif

namespace rlamd {

// Q fixed point for the shared (group_size > 1) mode where its range is proven:
// value = raw * 2^-QFRAC.
constexpr int QFRAC = 40;
// kinds of non-finite values (UCB + expected SARSA visible row flags, the f64
// representation's non-finite step contributions: IEEE sum algebra, order free)
constexpr uint32_t QF_NAN = 1u, QF_PINF = 2u, QF_NINF = 4u;
// replicas of the u64[8] stats block (same-address atomics from every block
// serialise; spreading them over replicas removed ~0.3 ms per launch)
constexpr uint32_t STATS_REP = 64;
// u64 words per stats replica: rl_stats slots 0-7 (slot 6, launches, is host-side),
// 8 = q_clamp_hits, 9 = delta_saturations
constexpr uint32_t STATS_W = 16;
constexpr uint32_t ACC_CLAMP = 8, ACC_SAT = 9;

// lane core record (uint4, SoA over lanes):
//   x = s (dense state), y = flags word below, z = env word (curr_step | blackjack hand),
//   w = training episodes finished in the current train() call
constexpr uint32_t LF_ACT_MASK = 0xffu;
constexpr uint32_t LF_NEED_RESET = 1u << 8;
constexpr uint32_t LF_READY = 1u << 9;
constexpr uint32_t LF_DFLAG = 1u << 10;   // DoubleTabularPolicy::policy_flag (starts true)
constexpr int LF_MODE_SHIFT = 12;         // rl_lane_mode, 2 bits
// lane aux record (uint4): x,y = epsilon (f64 bits), z = eval episodes left, w = episode length

// per-call Agent surface (rl_agent_get_action / rl_agent_update): device arrays
// of call_n entries, entry i for lane call_lane0 + i (dense states)
enum { CALL_NONE = 0, CALL_GET_ACTION = 1, CALL_UPDATE = 2 };
struct AgentCall {
    const uint32_t *s, *a, *s2, *a2;
    const double *r;
    const uint8_t *term;
    uint32_t *action_out;
    double *td_out;
};

struct KParams {
    uint32_t L, G, K, S, A, P;
    // per-call Agent surface (private mode): CALL_NONE for the training launches
    int32_t call_op;
    uint32_t call_lane0, call_n;
    AgentCall call;
    // lanes
    uint4 *core;
    uint4 *rng;
    uint4 *aux;
    double *epi_reward;
    // shared mode
    int64_t *q_base;       // [P][S][A]: fixed-point raw words, or f64 bits (fq)
    uint64_t *n_base;      // [S][A] UCB visit counts (u128 in the reference; u64 never wraps in practice)
    uint64_t *t_base;      // [1]
    int64_t *delta;        // the merge's SUM words: fixed point [P*S*A dq][P*S*A group counts][S*A dn][1 dt];
                           // f64 [psal grid sums][psal group counts][S*A dn][1 dt][3][psal kind counts]
    int64_t *delta_max;    // the merge's MAX words (f64: per-entry max code over the changed groups) [psal];
                           // the fixed point has none (delta == delta_max)
    int64_t *delta_rep;    // n_rep replicas of `delta`: group g adds into replica g % n_rep
    uint32_t n_rep;        // (spreads the same-address int64 atomics of the merge)
    uint32_t delta_words;  // replica stride (dense layout)
    uint32_t sum_words;    // SUM words in use: fixed point 2*PSA + SA + 1, f64 5*psal + SA + 1
    // f64 representation (rl_device.h "f64 shared Q"): every group writes its
    // final Q (LDS order, psal entries) to qslot[group][psal] for the merge
    int32_t fq;            // 1: shared Q is f64 (else the proven fixed point)
    int32_t trace_k;       // traces grid: 2^trace_k >= |lr| * trace bound (rl_host.cpp trace_grid_k)
    int32_t merge_hb;      // merge grid headroom bits (learner groups over every rank)
    uint32_t psal;         // LDS-held entries per group (Blackjack eps-greedy: compact rows)
    uint64_t *qslot;       // [n_groups][psal] f64 bits
    uint32_t n_groups;
    // private mode, LANE-MAJOR (round 5): a lane's table is one
    // contiguous block, so the row a step reads is one 16-byte-aligned run of A f64
    // (entry-major [entry][lane] put every lane's 8-byte gather in its own 128-B line)
    double *q_priv;        // [L][P][S][A]
    uint64_t *n_priv;      // [L][S*A]
    uint64_t *t_priv;      // [L]
    // eligibility traces, per lane a sparse set of the episode's visited states:
    // tlist[j] = j-th visited state, slot_of[s] = its slot (valid iff
    // slot_of[s] < tcnt && tlist[slot_of[s]] == s), trace[j*A + b] = E[tlist[j]][b]
    double *trace;         // [S*A][L] (slot-major)
    uint16_t *tlist;       // [S][L]
    uint16_t *slot_of;     // [S][L]
    uint32_t *tcnt;        // [L]
    // shared mode without UCB specials: the same buffers hold visited (state,
    // action) PAIRS instead — tlist[j] = pair id s*A+a | 0x8000 on the first pair
    // of its state, trace[j] = E of pair j.  During a launch the first slots live
    // in LDS (rl_train_impl.h PairCache); slot_of[s*A+a] and vbits (the visited
    // states) index the slots past them (layout_sparse_traces below)
    uint32_t *vbits;       // [ceil(S/32)][L]
    // Dyna (InternalModelAgent + RandomModel, private mode): per-lane model as a
    // sparse set in insertion order, entry j = (key = s*A+a, s', r)
    uint32_t plan_steps;
    uint32_t *mcnt;        // [L]
    uint4 *mrec;           // [L][S*A] entry j of a lane's model: {key = s*A+a, s', r lo, r hi} (16 B)
    uint32_t *mslot;       // [L][S*A] index + 1 of key in mrec, 0 = absent (cleared when the model empties)
    // NeuralPolicy (private mode): per-lane 2-layer MLP, parameters SoA [param][lane]
    // in the order [W1 n_in x H][b1 H][W2 H x A][b2 A] (rl.h rl_agent_net_dims)
    double *net_w;         // [n_params][L]
    const double *feat;    // [S][n_in] input-adapter features
    uint32_t n_in, n_hidden, n_params;
    int32_t act1, act2;    // rl_activation of the hidden / output layer
    // env tables
    const uint32_t *trans; // [S][A] packed
    const double *start_cdf;   // [n_start] running sums (categorical_sample); HBM
    uint32_t n_start;
    int32_t fixed_start;   // >= 0 when the start distribution is a single state
    int32_t slippery;      // FrozenLake with stochastic rows (else the per-step draw is skipped over)
    uint32_t max_steps;
    double th1, th2, th3;  // slippery FrozenLake cumulative sums
    double trunc_reward;
    // hyper-parameters
    double lr, gamma, gl, eps_decay, eps_final, ucb_c;
    // lr * 2^40 (exact): the fixed point's rint(RN(lr * td) * 2^40) is rint(RN(lr40 * td))
    // — scaling by 2^40 commutes with rounding; where lr * td is subnormal both are 0
    double lr40;
    double eps_dm, eps_ds;     // decay as eps * dm - ds (rl_device.h decay_eps)
    int32_t decay_kind, algo;  // algo: informational (kernels are specialised on it)
    // fixed point only: the host proved that a step's contributions to an entry fit
    // one int64 as sum * 2^11 + count (rl_host.cpp pack_proven): the 8-wave kernels
    // then use one LDS atomic each
    int32_t pack_ok;
    // UCB + expected SARSA: the launch's and the step's counter increments packed in
    // one u32 per entry (launch << 16 | step), possible while G * K < 2^16
    int32_t ucb_pack;
    // batched schedule option (rl_agent_set_reset_step; shared mode, eps-greedy):
    // a lane that needs a reset resets, selects and steps in one synchronous step
    int32_t reset_step;
    // train()/evaluate() control
    uint64_t target_episodes, eval_at;
    uint64_t eval_div;     // ceil(2^64 / eval_at) (mod 2^64): divisibility test constant
    uint32_t eval_episodes;
    int32_t eval_only;
    int32_t episodic;      // any of target_episodes / eval_at / eval_only set (else the run() fast path)
    // outputs
    unsigned long long *stats; // rl_stats as u64[STATS_W] x STATS_REP replicas (block b adds into b % STATS_REP)
    rl_step_record *rec;       // [K][L] or null
    rl_episode_record *elog;   // episode log [elog_cap][L] or null
    uint32_t *elog_cnt;        // [L] episodes logged per lane (ring position = cnt % elog_cap)
    uint32_t elog_cap;
    // Blackjack compact rows: terminal rows are never written (an update writes
    // Q[s] of a non-terminal s only), so they keep what reset / set_q stored.
    // When every terminal entry of table t holds one finite raw value bj_traw[t]
    // (the host checks at reset / set_q), the kernel uses it instead of a load.
    int32_t bj_tconst;
    int64_t bj_traw[2];
    // shared mode: lanes per wavefront (64; 32 / 16 spread a group over more
    // waves, host knob RLAMD_LPW): lane = group base + wave * lpw + lane-in-wave,
    // the other wave slots idle
    uint32_t lpw;
    uint32_t trc_kb;       // LDS KiB per learner group for pair-trace slots (rl_train_impl.h smem_layout)
    // private mode with small tables (round 5): lanes per wave of k_train_private_lds,
    // which holds its lanes' Q tables in LDS for the launch (0: k_train_private, Q in HBM)
    uint32_t priv_lpw;
    uint32_t net_regs;     // 1: NeuralPolicy lanes of the bin's network run k_train_private_net (rl_train_impl.h)
};

// one entry per (env, agent, policy, selector, private) kernel instantiation
// occ != nullptr: no launch; *occ = resident workgroups per CU of the kernel
// the launch would pick (hipOccupancyMaxActiveBlocksPerMultiprocessor)
typedef hipError_t (*train_launch_fn)(const KParams &p, dim3 grid, dim3 block, size_t smem,
                                      hipStream_t stream, int *occ);

// shared-mode traces sweep only the visited (state, action) pairs: an action
// never taken in a visited state has E = 0 and, with a finite td, contributes
// exactly 0 (it still counts toward its row's n).  UCB + expected SARSA can make
// td non-finite (0 * inf = NaN flags), so that variant keeps whole rows.
inline bool layout_sparse_traces(int agent, int sel, int algo, int priv) {
    return agent == RL_AGENT_TRACES && !priv && !(sel == RL_SEL_UCB && algo == RL_ALGO_EXPECTED_SARSA);
}
train_launch_fn lookup_train(int env, int agent, int policy, int sel, int algo, int priv);
size_t shared_smem_bytes(int env, int agent, int policy, int sel, int algo, uint32_t S, uint32_t A,
                         uint32_t n_start, uint32_t nthr, uint32_t trc_kb, int fq, int ucb_pack);
size_t private_smem_bytes(int env, int agent, int policy, int sel, uint32_t S, uint32_t A, uint32_t n_start);
// shared pair traces: LDS slots per lane for a carve, whether the env's lists use
// the HBM slot index, and its rebuild for a new slot count (rl_misc.hip)
uint32_t shared_pair_cap(int env, int agent, int policy, int sel, int algo, uint32_t S, uint32_t A,
                         uint32_t n_start, uint32_t nthr, uint32_t trc_kb, int fq, int ucb_pack);
bool pair_slot_index_env(int env);
void launch_pair_reindex(const KParams &p, uint32_t cap, hipStream_t s);
// the one-shot peer-read merge (rl_misc.hip k_peer_put / k_peer_reduce)
void launch_peer_put(const int64_t *src, int64_t *slot, uint64_t n, hipStream_t s);
void launch_peer_reduce(int64_t *const *bases, uint32_t world, uint32_t rank, uint64_t slot_off, uint64_t flag_off,
                        uint64_t n, int64_t epoch, int op_max, int64_t *dst, uint32_t *err, int64_t timeout_ticks,
                        hipStream_t s);
// the fixed point's merge over the peers in two launches (fold into the slot; reduce + apply)
void launch_peer_fold_put(const KParams &p, int64_t *slot, hipStream_t s);
void launch_peer_reduce_apply(const KParams &p, int64_t *const *bases, uint32_t world, uint32_t rank,
                              uint64_t slot_off, uint64_t flag_off, int64_t epoch, uint32_t *err,
                              int64_t timeout_ticks, hipStream_t s);

// env-only kernels (batched Env trait) and KAT probes
void launch_env_reset(int env, const KParams &p, hipStream_t s, uint64_t *obs);
void launch_env_step(int env, const KParams &p, hipStream_t s, const uint32_t *act, uint64_t *obs,
                     double *rew, uint8_t *term, unsigned int *not_ready);
void launch_lane_init(int env, const KParams &p, uint64_t seed, uint64_t lane_offset, double eps0,
                      hipStream_t s);
void launch_arm_full(const KParams &p, int32_t mode, uint32_t eval_left, int restore_eps, double eps0,
                     hipStream_t s);
void launch_fill_f64(double *ptr, uint64_t n, double v, hipStream_t s);
void launch_apply(const KParams &p, hipStream_t s);
// the f64 merge (rl_misc.hip): per entry max code / counts / kinds over the
// changed groups, then the grid sums, then base = their mean
void launch_fq_merge_a(const KParams &p, hipStream_t s);
void launch_fq_merge_b(const KParams &p, hipStream_t s);
void launch_fq_apply(const KParams &p, hipStream_t s);
void launch_fold_replicas(const KParams &p, hipStream_t s);
void launch_fold_apply(const KParams &p, hipStream_t s);
void launch_ctl_word(const KParams &p, int64_t *ctl, uint64_t lanes, int64_t status, hipStream_t s);
void launch_kat_log(const double *x, double *out, uint32_t n, hipStream_t s);
void launch_kat_rng(uint64_t seed, uint64_t lane, uint32_t n, uint32_t *out, hipStream_t s);
void launch_kat_ucb(const double *q, const double *nc, const uint64_t *t, double c, double *out,
                    uint32_t n, hipStream_t s);
void launch_kat_act(int act, const double *x, double *f, double *fp, uint32_t n, hipStream_t s);
// NeuralPolicy: DenseLayer::new / reset weights (gen 0 / >= 1) and get_values of every state
void launch_net_init(const KParams &p, uint64_t seed, uint64_t lane_offset, uint32_t gen, double scale1,
                     double low1, double scale2, double low2, hipStream_t s);
void launch_net_values(const KParams &p, double *out, hipStream_t s);

}  // namespace rlamd

/*
 * rlref.h — CPU ORACLE for the rl-rust_amd hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a plain-C restatement of JohnVithor/RL-Rust's tabular hot path
 * (reference @ /root/reference, cited as path:line).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
 * as the checker / CPU baseline — never as the product path.
 *
 * PARITY STATUS: "parity unpinned" in the strict sense.  The reference is Rust
 * (no rustc/cargo in this image), has no tests or fixtures (F2) and
 * draws from an entropy-seeded ChaCha12 ThreadRng (F3), so no reference output
 * can be reproduced.  What IS pinned: hand-derived known-answer tests taken
 * from the reference source (tests/golden/tables.json["kat"]), and an independent Python
 * construction restatement of every transition table (tests/golden/tables.json).
 * The RNG stream (xoshiro128+ per lane) replaces ThreadRng at exactly the
 * reference's draw sites, with rand-0.8.5's distribution mappings restated.
 *
 * Two restatements live here:
 *   1. rlo_faithful_*: one env + one agent, f64 Q, the control flow of
 *      src/agent.rs:66-141 line by line (train/evaluate, eval interleave,
 *      per-step training_error).  This is the "reference loop" and the
 *      cpu_baseline.
 *   2. rlo_batch_*: the batched schedule the GPU implements (learner groups of
 *      G lanes, snapshot semantics per synchronous step, int64 fixed-point Q,
 *      every entry moves by the MEAN of the deltas it received that step, and
 *      every K steps the base moves by the mean of the groups' changes).  G == 1 is the "private" mode: every lane is a
 *      whole reference agent with its own f64 Q / UCB counters and no merging,
 *      so lane i reproduces (1) seeded with lane id i BIT-EXACTLY.  (Fixed
 *      point at G=1 only tracks (1) until a near-tie flips an argmax: f64
 *      rounding order breaks exact ties that fixed point keeps.)
 */
#ifndef RLREF_H
#define RLREF_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { RLO_ENV_FROZEN_LAKE = 0, RLO_ENV_CLIFF_WALKING = 1, RLO_ENV_TAXI = 2, RLO_ENV_BLACKJACK = 3,
       RLO_ENV_FROZEN_LAKE_EDITED = 4 };
enum { RLO_AGENT_ONE_STEP = 0, RLO_AGENT_TRACES = 1 };
enum { RLO_POLICY_TABULAR = 0, RLO_POLICY_DOUBLE = 1, RLO_POLICY_NEURAL = 2 };
/* src/network/activation.rs */
enum { RLO_ACT_LINEAR = 0, RLO_ACT_TANH = 1, RLO_ACT_RELU = 2, RLO_ACT_LEAKY_RELU = 3, RLO_ACT_RELU6 = 4,
       RLO_ACT_LEAKY_RELU6 = 5, RLO_ACT_SIGMOID = 6, RLO_ACT_SOFTMAX = 7, RLO_ACT_SWISH = 8,
       RLO_ACT_HARD_SWISH = 9 };
enum { RLO_INPUT_SCALAR = 0, RLO_INPUT_FL_OBS = 1 };
enum { RLO_SEL_EPS_GREEDY = 0, RLO_SEL_UCB = 1 };
enum { RLO_ALGO_SARSA = 0, RLO_ALGO_QLEARNING = 1, RLO_ALGO_EXPECTED_SARSA = 2 };
enum { RLO_DECAY_LINEAR = 0, RLO_DECAY_MUL = 1 };
enum { RLO_MODE_TRAIN = 0, RLO_MODE_EVAL = 1, RLO_MODE_DONE = 2 };

/* Q fixed point: value = q_raw * 2^-RLO_QFRAC (batched schedule only). */
#define RLO_QFRAC 40

typedef struct {
    int32_t env, map8x8, slippery;
    uint32_t max_steps;
    int32_t agent, policy, selector, algo, decay_kind;
    double lr, gamma, lambda_, eps0, eps_decay, eps_final, ucb_c, q_default;
    uint64_t seed;
    uint64_t lane_offset;     /* global id of local lane 0 (multi-GPU sharding) */
    uint32_t n_lanes, group_size, sync_every;
    uint32_t eval_episodes;   /* episodes per in-train evaluate() call (reference: 100) */
    /* NeuralPolicy (policy == RLO_POLICY_NEURAL): DenseLayer(n_in, hidden) -> act1 ->
     * DenseLayer(hidden, A) -> act2, mse loss (src/bin/frozen_lake_neural.rs:130-134) */
    int32_t net_input;        /* RLO_INPUT_* */
    uint32_t net_hidden;
    int32_t net_act1, net_act2;
} rlo_config;

/* one per-lane-per-step record (same layout as the product's rl_step_record).
 * kind: 0 idle (lane done), 1 RESET (s, a = new episode's state and first
 * action), 2 STEP (s, a, r, term, s2, a2, td) */
typedef struct {
    uint32_t s, s2;
    uint8_t a, a2, term, mode;
    uint8_t kind, pad[3];
    double r, td;
} rlo_record;

/* ---------------- primitives (exported for known-answer tests) ---------------- */
double   rlo_log(double x);                         /* fdlibm-style ln shared definition */
void     rlo_rng_stream(uint64_t seed, uint64_t lane, uint32_t n, uint32_t *out);
double   rlo_u64_to_uniform01(uint64_t bits);       /* rand 0.8 UniformFloat<f64>(0..1) */
uint32_t rlo_uniform_int_u64(uint64_t v, uint64_t range, int *reject);  /* rand 0.8 UniformInt<usize> */
uint32_t rlo_uniform_card_u32(uint32_t v, int *reject);                 /* rand 0.8 Uniform<u8>(1..11) */
uint32_t rlo_uniform_card_u16(uint32_t h, int *reject);                 /* the stream's card rule on a 16-bit half */
int rlo_eps_test_words(uint32_t h, uint32_t l, double eps, int *need_low); /* the stream's eps test (l read only if *need_low) */
uint64_t rlo_blackjack_obs_id(uint32_t p_score, uint32_t d_score, uint32_t p_ace); /* fxhash 0.2.1 */
int      rlo_env_dims(const rlo_config *c, uint32_t *n_states, uint32_t *n_actions);
/* transition table export: for each (s,a) up to 3 outcomes (prob, next, reward, term) */
int      rlo_env_table(const rlo_config *c, double *prob, uint32_t *next, double *reward, uint8_t *term);
int      rlo_env_start(const rlo_config *c, double *start);   /* initial-state distribution */
/* Env::reset then Env::step(actions[i]) for i < n on the stream (seed, lane);
 * writes s0 then per step (s', r, term); returns steps taken before EnvNotReady
 * (a step after termination stops the walk), -1 on bad config */
int      rlo_env_walk(const rlo_config *c, uint64_t lane, uint32_t n, const uint32_t *actions,
                      uint32_t *s0, uint32_t *s_next, double *reward, uint8_t *term);

/* fdlibm e_exp / s_expm1 / s_tanh operation sequences (shared with the device) */
double   rlo_exp(double x);
double   rlo_expm1(double x);
double   rlo_tanh(double x);
/* activation f(x), f'(x) (src/network/activation.rs); not RLO_ACT_SOFTMAX */
void     rlo_act(int32_t act, double x, double *f, double *fprime);
/* network sizes for a config: input features and per-agent parameter count
 * ([W1 n_in x H][b1 H][W2 H x A][b2 A]); -1 if the config has no valid network */
int      rlo_net_dims(const rlo_config *c, uint32_t *n_in, uint32_t *n_params);
/* input-adapter features of every dense state, [S][n_in] */
int      rlo_net_features(const rlo_config *c, double *out);
/* DenseLayer::new (gen 0: bias 0) / DenseLayer::reset (gen >= 1: bias 0.1) weights of
 * the agent on lane `lane` (layers.rs:59-73, :90-95) */
void     rlo_net_init(const rlo_config *c, uint64_t lane, uint32_t gen, double *w);
/* Network::predict (src/network.rs:51-58): y = act2(W2' act1(W1' x + b1) + b2) */
void     rlo_net_forward(const rlo_config *c, const double *w, const double *x, double *y);
/* Network::fit (src/network.rs:61-80), one sample, plain SGD at rate lr */
void     rlo_net_fit(const rlo_config *c, double *w, const double *x, const double *y_target, double lr);

/* rand 0.8.5 gen_range(0..range) for usize (sample_single_inclusive): index + reject flag */
uint64_t rlo_gen_index_u64(uint64_t v, uint64_t range, int *reject);

/* ---------------- faithful single-env restatement (f64) ---------------- */
typedef struct rlo_faithful rlo_faithful;
rlo_faithful *rlo_faithful_create(const rlo_config *c);
void   rlo_faithful_destroy(rlo_faithful *f);
/* Agent::train(env, n_episodes, eval_at) (src/agent.rs:66-118).  Histories are
 * appended to internal buffers; returns the number of training steps. */
uint64_t rlo_faithful_train(rlo_faithful *f, uint64_t n_episodes, uint64_t eval_at);
uint64_t rlo_faithful_evaluate(rlo_faithful *f, uint64_t n_episodes);
void   rlo_faithful_reset(rlo_faithful *f);                     /* Agent::reset */
void   rlo_faithful_get_q(const rlo_faithful *f, double *out);  /* P*S*A */
uint64_t rlo_faithful_n_episodes(const rlo_faithful *f);
uint64_t rlo_faithful_n_steps(const rlo_faithful *f);
void   rlo_faithful_histories(const rlo_faithful *f, double *reward_history,
                              uint64_t *episode_length, double *training_error);
/* per-step integer stream of the last train() call (s, a, r, term, s2, a2) */
uint64_t rlo_faithful_get_records(const rlo_faithful *f, rlo_record *out, uint64_t cap);
void   rlo_faithful_set_record(rlo_faithful *f, int enable);
double rlo_faithful_epsilon(const rlo_faithful *f);
/* NeuralPolicy parameters (n_params doubles) */
void   rlo_faithful_get_weights(const rlo_faithful *f, double *out);
void   rlo_faithful_set_weights(rlo_faithful *f, const double *in);
/* InternalModelAgent::new(agent, RandomModel::default(), planning_steps)
 * (src/agent/internal_model_agent.rs:20-31); 0 = the plain agent */
void   rlo_faithful_set_planning(rlo_faithful *f, uint32_t planning_steps);
/* the bench cpu baseline: train for `budget_steps` env steps and return the
 * steps actually run (whole episodes), no recording */
uint64_t rlo_faithful_bench(const rlo_config *c, uint64_t n_episodes, uint64_t eval_at,
                            double *seconds);

/* ---------------- batched schedule (fixed-point, the GPU semantics) ---------------- */
typedef struct rlo_batch rlo_batch;
rlo_batch *rlo_batch_create(const rlo_config *c);
void   rlo_batch_destroy(rlo_batch *b);
/* one launch split for multi-rank use: run local groups, ADD their changes to
 * `delta` (GPU layout, rlo_batch_delta_words int64), then apply the (all-reduced) total */
uint64_t rlo_batch_delta_words(const rlo_batch *b);
void   rlo_batch_launch_groups(rlo_batch *b, int64_t *delta);
void   rlo_batch_apply_delta(rlo_batch *b, const int64_t *delta);
/* run `n_launches` launches of K = sync_every synchronous steps each */
void   rlo_batch_run(rlo_batch *b, uint32_t n_launches);
/* Agent::train for every lane: launches until every lane has finished n_episodes
 * training episodes (+ pending eval); returns number of launches */
uint64_t rlo_batch_train_episodes(rlo_batch *b, uint64_t n_episodes, uint64_t eval_at);
uint64_t rlo_batch_evaluate(rlo_batch *b, uint64_t n_episodes);
void   rlo_batch_reset(rlo_batch *b);
/* shared mode (G >= 2): [P][S][A] merged base; private mode (G == 1): [L][P][S][A] f64
 * (NeuralPolicy: Policy::get_values of every state, [L][1][S][A]) */
void   rlo_batch_get_q(const rlo_batch *b, double *out);
void   rlo_batch_get_q_raw(const rlo_batch *b, int64_t *out);   /* P*S*A raw fixed point */
void   rlo_batch_set_q(rlo_batch *b, const double *in);         /* shared P*S*A / private [L][P][S][A] */
void   rlo_batch_get_qflags(const rlo_batch *b, uint8_t *out);
void   rlo_batch_get_ucb(const rlo_batch *b, uint64_t *counts, uint64_t *t);
void   rlo_batch_set_ucb(rlo_batch *b, const uint64_t *counts, const uint64_t *t);
void   rlo_batch_set_record(rlo_batch *b, int enable);
/* records of all steps since the last call, laid out [step][lane] */
uint64_t rlo_batch_take_records(rlo_batch *b, rlo_record *out, uint64_t cap);
uint64_t rlo_batch_n_records(const rlo_batch *b);
void   rlo_batch_stats(const rlo_batch *b, uint64_t *out16);   /* rl_stats order, see rlref.c */
void   rlo_batch_lane_eps(const rlo_batch *b, double *out);
/* NeuralPolicy parameters of every lane, [L][n_params] */
void   rlo_batch_get_weights(const rlo_batch *b, double *out);
void   rlo_batch_set_weights(rlo_batch *b, const double *in);
void   rlo_batch_set_selector(rlo_batch *b, int32_t selector);
void   rlo_batch_set_algo(rlo_batch *b, int32_t algo);
/* Dyna planning steps per update (private mode only; -1 otherwise) */
int    rlo_batch_set_planning(rlo_batch *b, uint32_t planning_steps);
/* batched schedule option: a lane needing a reset resets, selects (snapshot) and
 * steps in the same synchronous step (record kind 3); shared mode, eps-greedy */
void   rlo_batch_set_reset_step(rlo_batch *b, int on);
/* shared-Q representation (rlref.c section 2): the int64 fixed point only where
 * the range proof holds, else f64 with the reference's full range */
enum { RLO_QREPR_FIXED40 = 0, RLO_QREPR_F64 = 1, RLO_QREPR_PRIVATE = 2 };
enum { RLO_QMODE_AUTO = 0, RLO_QMODE_F64 = 1, RLO_QMODE_F64_SEQ = 2, RLO_QMODE_FIXED_RANGE = 3 };
void   rlo_batch_set_q_mode(rlo_batch *b, int mode);
int    rlo_batch_q_repr(const rlo_batch *b);
/* learner groups over every rank (the f64 merge grid's headroom); 0 = local */
void   rlo_batch_set_merge_groups(rlo_batch *b, uint64_t total_groups);
/* merge buffer: the first rlo_batch_delta_max_words words are all-reduced with MAX
 * before rlo_batch_fold, the rest with SUM before rlo_batch_apply_delta */
uint64_t rlo_batch_delta_max_words(const rlo_batch *b);
void   rlo_batch_fold(rlo_batch *b, int64_t *delta);
/* traces grid exponent (rlref.c rlo_trace_grid_k) */
int    rlo_trace_grid_k(double lr, double gamma, double lambda_, uint32_t max_steps, int32_t env);

#ifdef __cplusplus
}
#endif
#endif

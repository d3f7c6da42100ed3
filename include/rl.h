/*
 * rl.h — C ABI of librlamd.so, the MI355X-native (gfx950, HIP) tabular-RL hot path.
 *
 * This is the drop-in boundary for JohnVithor/RL-Rust's per-step training loop
 * (reference: /root/reference, cited path:line).  The reference has no FFI;
 * its interfaces are Rust traits:
 *   Env<T,COUNT>            src/env.rs:19-49
 *   Agent<T,COUNT>          src/agent.rs:47-164
 *   Policy<T,COUNT>         src/policy.rs:15-33          (EnumPolicy)
 *   ActionSelection<T,COUNT> src/action_selection.rs:10-22 (EnumActionSelection)
 *   GetNextQValue fn ptr    src/agent.rs:17  (sarsa / qlearning / expected_sarsa)
 * Each export below names the trait method it replaces.  Closures and fn
 * pointers become enums; every Env/Agent is BATCHED over `n_lanes` lanes
 * (lane = one env instance + its RNG stream).  The Rust binding a maintainer
 * would add is shown in INTEGRATION.md.
 *
 * Ownership: a handle owns all its device memory; host buffers passed in are
 * owned by the caller and only read/written during the call.  Sizes are
 * explicit.  No callbacks, no C++ exceptions cross this boundary.  One handle
 * per host thread (not thread-safe), like the reference's !Send agents.
 * Errors: every int-returning call returns RL_OK or an RL_E_* code; the
 * message is in rl_last_error().  EnvNotReady (src/env.rs:17) is RL_E_NOT_READY.
 */
#ifndef RL_AMD_RL_H
#define RL_AMD_RL_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RL_ABI_VERSION 7

enum rl_status {
    RL_OK = 0,
    RL_E_NOT_READY = 1, /* Env::step on a terminated/unreset env (src/env.rs:16-17,24) */
    RL_E_ARG = 2,       /* invalid argument / size */
    RL_E_HIP = 3,       /* HIP runtime failure */
    RL_E_OOM = 4,       /* device allocation failed */
    RL_E_STATE = 5,     /* call not valid in the handle's current mode */
    RL_E_RCCL = 6       /* RCCL (collective) failure */
};

enum rl_env_kind {      /* src/env/{frozen_lake,cliff_walking,taxi,blackjack,frozen_lake_edited}.rs */
    RL_ENV_FROZEN_LAKE = 0, RL_ENV_CLIFF_WALKING = 1, RL_ENV_TAXI = 2, RL_ENV_BLACKJACK = 3,
    RL_ENV_FROZEN_LAKE_EDITED = 4   /* FrozenLakeEditedEnv: obs = FrozenLakeObs, dense index = position */
};
enum rl_agent_kind {    /* src/agent/one_step_agent.rs, src/agent/elegibility_traces_agent.rs */
    RL_AGENT_ONE_STEP = 0, RL_AGENT_TRACES = 1
};
enum rl_policy_kind {   /* src/policy/{tabular_policy,double_tabular_policy,neural_policy}.rs */
    RL_POLICY_TABULAR = 0, RL_POLICY_DOUBLE = 1,
    RL_POLICY_NEURAL = 2    /* NeuralPolicy over a 2-layer Network (src/policy/neural_policy.rs,
                               src/network/); private mode (group_size 1) only */
};
/* Network activations (src/network/activation.rs); the pair (f, f') of each.
 * RL_ACT_SOFTMAX normalises the whole layer and is accepted for the output layer only. */
enum rl_activation {
    RL_ACT_LINEAR = 0, RL_ACT_TANH = 1, RL_ACT_RELU = 2, RL_ACT_LEAKY_RELU = 3, RL_ACT_RELU6 = 4,
    RL_ACT_LEAKY_RELU6 = 5, RL_ACT_SIGMOID = 6, RL_ACT_SOFTMAX = 7, RL_ACT_SWISH = 8,
    RL_ACT_HARD_SWISH = 9
};
/* NeuralPolicy input adapters (InputAdapter<T> = fn(T) -> Array2<f64>, neural_policy.rs:9) */
enum rl_input_adapter {
    RL_INPUT_SCALAR = 0,  /* [[obs as f64]] of the reference's usize observation
                             (src/bin/frozen_lake_neural.rs:147-149) */
    RL_INPUT_FL_OBS = 1   /* [left, down, right, up terrain values, x, y] of FrozenLakeObs
                             (frozen_lake_neural.rs:136-145; values frozen_lake_edited.rs:18-28);
                             FrozenLake / FrozenLakeEdited only */
};
enum rl_selector_kind { /* src/action_selection/{uniform_epsilon_greed,upper_confidence_bound}.rs */
    RL_SEL_EPS_GREEDY = 0, RL_SEL_UCB = 1
};
enum rl_algo_kind {     /* src/agent.rs:19-45 sarsa / qlearning / expected_sarsa */
    RL_ALGO_SARSA = 0, RL_ALGO_QLEARNING = 1, RL_ALGO_EXPECTED_SARSA = 2
};
enum rl_decay_kind {    /* the epsilon_decay closure: `a - d` (src/bin/frozen_lake.rs:146) or `a * d`
                           (src/bin/frozen_lake_neural.rs:181) */
    RL_DECAY_LINEAR = 0, RL_DECAY_MUL = 1
};
enum rl_lane_mode { RL_MODE_TRAIN = 0, RL_MODE_EVAL = 1, RL_MODE_DONE = 2 };
/* How a shared-mode (group_size > 1) Q table is held (rl_agent_q_repr):
 *   RL_QREPR_FIXED40: int64 fixed point, value = raw * 2^-40 — only where the
 *       host proves |Q| stays within 2048 (one-step agent, single table, a
 *       bootstrap that is a sub-convex combination of Q values: SARSA, Q-learning,
 *       expected SARSA over eps-greedy), so no update is ever clamped;
 *   RL_QREPR_F64: the reference's f64 with its whole range (+-inf, NaN included:
 *       the double policy's A - B grows by (1 + lr) per update pair,
 *       double_tabular_policy.rs:50-57; UCB + expected SARSA reaches NaN);
 *   RL_QREPR_PRIVATE: group_size 1, each lane an f64 reference agent.
 * A step's simultaneous contributions to one entry are combined order-free:
 * their mean, with the sum formed exactly on the integer grid of the largest
 * one.  One contribution of a one-step agent is exactly Q += lr * td
 * (tabular_policy.rs:35-38).  Two exceptions: eligibility traces
 * round every lr * (td * E) of a group step onto one grid per step, 2^(code of the
 * step's largest |td| - 1075 + trace_k), so a single-lane shared traces agent
 * differs from the reference loop at about 1e-13 relative (private mode,
 * group_size 1, is the reference loop bit for bit); and when the learner groups
 * over every rank exceed 1024, the merge grid gives up ceil(log2(groups)) - 10
 * low bits of headroom, also for entries only one group changed. */
enum rl_q_repr { RL_QREPR_FIXED40 = 0, RL_QREPR_F64 = 1, RL_QREPR_PRIVATE = 2 };
enum rl_q_mode {        /* rl_agent_set_q_mode */
    RL_QMODE_AUTO = 0,  /* the fixed point where proven (and the table is exact in it), else f64 */
    RL_QMODE_F64 = 1    /* f64 always */
};

/* Env constructor arguments: FrozenLakeEnv::new(map, is_slippery, max_steps)
 * (src/env/frozen_lake.rs:48), CliffWalkingEnv::new(max_steps) (cliff_walking.rs:34),
 * TaxiEnv::new(max_steps) (taxi.rs:57), BlackJackEnv::new() (blackjack.rs:32). */
typedef struct rl_env_config {
    int32_t kind;       /* rl_env_kind */
    int32_t map8x8;     /* FrozenLake: 0 = MAP_4X4, 1 = MAP_8X8 (frozen_lake.rs:23-28) */
    int32_t slippery;   /* FrozenLake --stochastic_env */
    uint32_t max_steps; /* truncation (frozen_lake.rs:119); ignored by Blackjack */
} rl_env_config;

/* NeuralPolicy::new(lr, input_adapter, network, output_adapter, inv_output_adapter)
 * (src/policy/neural_policy.rs:20-35) with the bin's network shape
 * (src/bin/frozen_lake_neural.rs:130-134): DenseLayer(n_in, hidden) -> act_hidden ->
 * DenseLayer(hidden, COUNT) -> act_out, loss mse/mse_prime (src/network/loss.rs).
 * The output adapters are the identity on COUNT values.  Ignored unless
 * policy == RL_POLICY_NEURAL.  hidden <= RL_NET_MAX_HIDDEN. */
#define RL_NET_MAX_HIDDEN 256
#define RL_NET_MAX_INPUT 8
typedef struct rl_network_config {
    int32_t input;        /* rl_input_adapter */
    uint32_t hidden;      /* 32 in the bin */
    int32_t act_hidden;   /* rl_activation, RL_ACT_LEAKY_RELU6 in the bin */
    int32_t act_out;      /* rl_activation, RL_ACT_LINEAR in the bin */
} rl_network_config;

/* Agent constructor arguments, gathered from the bins (src/bin/frozen_lake.rs:140-165):
 * OneStepAgent::new / ElegibilityTracesAgent::new + TabularPolicy::new(lr, default)
 * + UniformEpsilonGreed::new(eps0, decay, final) | UpperConfidenceBound::new(c). */
typedef struct rl_agent_config {
    rl_env_config env;
    int32_t agent, policy, selector, algo, decay_kind;
    double lr, gamma, lambda, eps0, eps_decay, eps_final, ucb_c, q_default;
    uint64_t seed;        /* per-lane RNG key (replaces thread_rng) */
    uint64_t lane_offset; /* global id of local lane 0 (multi-GPU sharding) */
    uint32_t n_lanes;     /* env instances on this device */
    uint32_t group_size;  /* lanes sharing one Q copy; 1 = private f64 agents (bit-exact reference) */
    uint32_t sync_every;  /* K: synchronous steps per launch; groups merge after every launch */
    uint32_t eval_episodes; /* episodes per in-train evaluate() (src/agent.rs:108 uses 100) */
    int32_t device;       /* HIP device ordinal */
    rl_network_config net; /* policy == RL_POLICY_NEURAL only */
} rl_agent_config;

/* One per lane per synchronous step (recording mode only).  A live lane does
 * one of two things per step (src/agent.rs:83-106 cut at its get_action calls):
 *   kind 1 RESET: s = Env::reset(), a = get_action(s)              (s, a set)
 *   kind 2 STEP:  (s2, r, term) = Env::step(a), a2 = get_action(s2), update;
 *                 td is the value pushed to training_error (src/agent.rs:98)
 *   kind 3 RESET + STEP (rl_agent_set_reset_step): s = Env::reset(), a =
 *                 get_action(s), then kind 2 from (s, a)
 *   kind 0: lane idle (finished its train()/evaluate() call)
 * For Blackjack s/s2 are dense indices (p_score*32 + d_score)*2 + p_ace (S = 2048;
 * see rl_obs_to_reference). */
typedef struct rl_step_record {
    uint32_t s, s2;
    uint8_t a, a2, term, mode;
    uint8_t kind, pad[3];
    double r, td;
} rl_step_record;

/* One per finished episode (episode log only): the reward_history /
 * episode_length entries of Agent::train / Agent::evaluate (src/agent.rs:72-141).
 * seq = the lane's running episode-log index (train and eval episodes interleaved
 * in the order they finished); mode = RL_MODE_TRAIN or RL_MODE_EVAL. */
typedef struct rl_episode_record {
    uint32_t lane, length, seq;
    uint8_t mode, pad[3];
    double reward;
} rl_episode_record;

/* Counters accumulated since rl_agent_create. */
typedef struct rl_stats {
    uint64_t train_steps;     /* every Env::step inside train, truncation step included */
    uint64_t eval_steps;      /* steps of in-train evaluate() episodes (excluded from the metric) */
    uint64_t train_episodes;
    uint64_t eval_episodes;
    int64_t reward_sum_q16;   /* sum of training-episode rewards, fixed point 2^-16 */
    uint64_t done_lanes;      /* lanes that finished the current train()/evaluate() call */
    uint64_t launches;        /* train launches queued; each train() / evaluate() call counts
                                 one launch past its last working one (the exit test reads
                                 the control word one launch behind; that launch is a no-op) */
    uint64_t trace_states;    /* traces agents: sum over training steps of the visited-set size
                                 swept by the eligibility update (mean = V-bar of SURVEY 8(d)) */
    /* ABI v3 counted updates clamped to a fixed-point range; since v4 no range is
     * ever clamped (rl_q_repr), so q_clamp_hits stays 0.  delta_saturations counts
     * f64 merge entries changed by more learner groups than the merge grid's
     * headroom allows (more than rl_agent_set_merge_groups declared, external
     * collectives only): such a merge is not exact, and train / evaluate return
     * RL_E_STATE when it happens */
    uint64_t q_clamp_hits;
    uint64_t delta_saturations;
} rl_stats;

typedef struct rl_env rl_env;
typedef struct rl_agent rl_agent;
typedef struct rl_comm rl_comm;

/* ---------------------------------------------------------------- misc */
const char *rl_last_error(void);
int rl_abi_version(void);
/* how this librlamd.so was built: compiler flags, target, experiment switches, build id */
const char *rl_build_info(void);
/* "src:<16 hex> git:<12 hex>": the first 16 hex digits of the sha256 of every
 * source the library was built from (rl-rust_amd/Makefile ID_SRCS, in that order)
 * and the git HEAD at link time.  Profiles and bench lines carry it, so numbers
 * can be matched to the binary that produced them. */
const char *rl_build_id(void);
int rl_device_count(int *count);
/* usize observation id of the reference's Blackjack env: fxhash 0.2.1 of
 * BlackJackObservation{p_score,d_score,p_ace} (src/env/blackjack.rs:25-27). */
uint64_t rl_blackjack_obs_id(uint32_t p_score, uint32_t d_score, uint32_t p_ace);
/* dense state index <-> reference observation (Blackjack: fxhash id; others: identity) */
uint64_t rl_obs_to_reference(int32_t env_kind, uint32_t dense_state);
/* the inverse: a reference observation (usize; Blackjack: its fxhash id) as the
 * dense state index; RL_E_ARG when it is none of the env's observations */
int rl_obs_from_reference(int32_t env_kind, uint64_t obs, uint32_t *dense_state);
/* |S| and COUNT (Env::action_size, src/env.rs:20-22) for an env config */
int rl_env_dims(const rl_env_config *cfg, uint32_t *n_states, uint32_t *n_actions);
/* Host-side export of the packed device transition tables, decoded to the
 * reference's layout probs[s][a][3] = (p, s', r, term) (frozen_lake.rs:56,
 * cliff_walking.rs:12, taxi.rs:14) plus the initial-state distribution.
 * Needs no GPU.  Not available for Blackjack (no table). */
int rl_env_table(const rl_env_config *cfg, double *prob, uint32_t *next, double *reward,
                 uint8_t *term, double *start);

/* ---------------------------------------------------------------- Env (batched) */
/* Env::new for n_envs lanes; lane i draws from stream (seed, lane_offset + i). */
int rl_env_create(const rl_env_config *cfg, uint32_t n_envs, uint64_t seed, uint64_t lane_offset,
                  int32_t device, rl_env **out);
void rl_env_destroy(rl_env *env);
/* Env::reset (src/env.rs:23) for every lane: obs_out[n_envs] (usize observations) */
int rl_env_reset(rl_env *env, uint64_t *obs_out);
/* Env::step (src/env.rs:24) for every lane.  Returns RL_E_NOT_READY (and steps
 * no lane) if any lane is not ready — the batched Err(EnvNotReady). */
int rl_env_step(rl_env *env, const uint32_t *actions, uint64_t *obs_out, double *reward_out,
                uint8_t *terminated_out);

/* One lane's Env::reset / Env::step (the reference's single env, src/env.rs:23-24):
 * RL_E_NOT_READY when that lane terminated and was not reset; the other lanes are
 * untouched.  `action` as usize, obs as the reference's usize id. */
int rl_env_reset_lane(rl_env *env, uint32_t lane, uint64_t *obs);
int rl_env_step_lane(rl_env *env, uint32_t lane, uint32_t action, uint64_t *obs, double *reward,
                     uint8_t *terminated);

/* ---------------------------------------------------------------- Agent (batched) */
int rl_agent_create(const rl_agent_config *cfg, rl_agent **out);
void rl_agent_destroy(rl_agent *a);
/* Agent::set_future_q_value_func (src/agent.rs:48) */
int rl_agent_set_future_q_value_func(rl_agent *a, int32_t algo);
/* Agent::set_action_selector (src/agent.rs:50) with a freshly constructed selector */
int rl_agent_set_action_selector(rl_agent *a, int32_t selector, double eps0, double eps_decay,
                                 double eps_final, int32_t decay_kind, double ucb_c);
/* Agent::reset (one_step_agent.rs:43-46): policy to default, selector fresh */
int rl_agent_reset(rl_agent *a);
/* Agent::train(env, n_episodes, eval_at) (src/agent.rs:66-118) for every lane:
 * returns when every lane has run n_episodes training episodes (eval_at = 0
 * disables the evaluate() interleave; the reference panics on 0). */
int rl_agent_train(rl_agent *a, uint64_t n_episodes, uint64_t eval_at, rl_stats *out);
/* Agent::evaluate(env, n_episodes) (src/agent.rs:120-141) for every lane */
int rl_agent_evaluate(rl_agent *a, uint64_t n_episodes, rl_stats *out);
/* ---- the per-call Agent surface: the required methods of trait Agent
 * (src/agent.rs:52-62) on one lane's agent, so that `impl Agent<usize, COUNT> for
 * GpuAgent` exists and the reference's default train / evaluate
 * (src/agent.rs:66-141) and the bins' direct loops (src/bin/blackjack.rs:183-200)
 * run over it unchanged.  Private mode (group_size 1) only: every lane is a whole
 * reference agent (RL_E_STATE otherwise).  Observations are the reference's usize
 * ids (Blackjack: the fxhash id, rl_obs_to_reference), as rl_env_reset / step return
 * them.  The selector's draws come from the lane's RNG stream; an Env view of the
 * same agent (rl_agent_env) draws the env's from that same stream, which is how
 * the reference's one thread_rng serves both.  Each call is one kernel launch and
 * one round trip: the compatibility path, not the throughput one (rl_agent_train). */
/* Agent::get_action(&obs) (src/agent.rs:52; one_step_agent.rs:48-51): ε-greedy
 * draws / UCB counter increments happen as in the reference */
int rl_agent_get_action(rl_agent *a, uint32_t lane, uint64_t obs, uint32_t *action);
/* Agent::update(curr_obs, curr_action, reward, terminated, next_obs, next_action)
 * (src/agent.rs:54-62; one_step_agent.rs:53-86, elegibility_traces_agent.rs:61-104,
 * internal_model_agent.rs:47-77 when planning is on): *td = the TD error it returns */
int rl_agent_update(rl_agent *a, uint32_t lane, uint64_t curr_obs, uint32_t curr_action, double reward,
                    int32_t terminated, uint64_t next_obs, uint32_t next_action, double *td);
/* the same two for every lane at once (arrays of n_lanes entries; lane i is agent i).
 * ABI 6: n_lanes is the caller's array length and must equal the agent's lane
 * count (RL_E_ARG otherwise), so the library never reads past a shorter array */
int rl_agent_get_actions(rl_agent *a, const uint64_t *obs, uint32_t *actions, uint64_t n_lanes);
int rl_agent_updates(rl_agent *a, const uint64_t *curr_obs, const uint32_t *curr_action, const double *reward,
                     const uint8_t *terminated, const uint64_t *next_obs, const uint32_t *next_action, double *td,
                     uint64_t n_lanes);
/* An Env over the agent's own lanes (one env per lane, the agent's RNG streams and
 * tables, the agent's stream): rl_env_reset / rl_env_step on it are Env::reset /
 * Env::step of the lane's env.  One view per agent; destroy it (rl_env_destroy)
 * before the agent.  train / evaluate start every lane at a fresh reset, so the
 * per-call and the batched loops can be mixed on one agent. */
int rl_agent_env(rl_agent *a, rl_env **out);

/* Throughput mode: enqueue n launches of K = sync_every synchronous steps over
 * all lanes (lanes train forever, episodes restart), each followed by the group
 * merge.  Asynchronous on the handle's stream. */
int rl_agent_run(rl_agent *a, uint32_t n_launches);
int rl_agent_synchronize(rl_agent *a);
int rl_agent_stats(rl_agent *a, rl_stats *out);
/* Policy::get_values for every (s,a): shared mode (group_size>1): [P][S][A]
 * merged Q; private mode (group_size==1): [n_lanes][P][S][A].  P = 2 for the
 * double policy (alpha, beta).  n = number of doubles in out. */
int rl_agent_get_q(rl_agent *a, double *out, size_t n);
int rl_agent_set_q(rl_agent *a, const double *in, size_t n);
/* shared mode only: the raw words of Q — the fixed-point integers (value = raw *
 * 2^-40) or the f64 bits (NaN canonical 0x7FF8000000000000), per rl_agent_q_repr */
int rl_agent_get_q_raw(rl_agent *a, int64_t *out, size_t n);
/* the shared Q representation now (rl_q_repr) */
int rl_agent_q_repr(rl_agent *a, int32_t *repr);
/* request a representation (rl_q_mode).  Switching to f64 is exact; AUTO goes
 * back to the fixed point only when the proof holds and every value is exact in it. */
int rl_agent_set_q_mode(rl_agent *a, int32_t mode);
/* UCB counters (upper_confidence_bound.rs:11-12, u128 there; u64 here: 2^64
 * selections of one entry is out of reach): shared [S][A] + t[1];
 * private [n_lanes][S][A] + t[n_lanes] */
int rl_agent_get_ucb(rl_agent *a, uint64_t *counts, size_t n_counts, uint64_t *t, size_t n_t);
/* set the UCB counters (same layout; t >= 1), e.g. to resume a checkpoint */
int rl_agent_set_ucb(rl_agent *a, const uint64_t *counts, size_t n_counts, const uint64_t *t, size_t n_t);
/* per-lane epsilon (UniformEpsilonGreed::epsilon, uniform_epsilon_greed.rs:13) */
int rl_agent_get_epsilon(rl_agent *a, double *out, size_t n);
/* recording: every launch appends K*n_lanes rl_step_record ([step][lane]) */
int rl_agent_set_recording(rl_agent *a, int32_t enable);
int rl_agent_take_records(rl_agent *a, rl_step_record *out, uint64_t cap, uint64_t *n_total);
int rl_agent_dims(rl_agent *a, uint32_t *n_states, uint32_t *n_actions, uint32_t *n_tables);
/* InternalModelAgent::new(agent, RandomModel::default(), planning_steps)
 * (src/agent/internal_model_agent.rs:20-31, src/model/random_model.rs): Dyna
 * planning after every training update; 0 = the plain agent.  Private mode
 * (group_size 1) only; the model is emptied here and by rl_agent_reset. */
int rl_agent_set_planning(rl_agent *a, uint32_t planning_steps);
/* Batched-schedule option (shared mode, eps-greedy selection; no reference
 * counterpart — the reference has one env): off (default), a lane that needs a
 * reset spends a synchronous step on env.reset() + get_action (kind 1 record);
 * on, it resets, selects AND steps in the same synchronous step (one kind 3
 * record: a STEP whose (s, a) came from the reset), both selections reading the
 * step's Q snapshot.  Each lane still runs the reference loop (src/agent.rs:80-106)
 * in order; worth it where episodes are short (Blackjack: ~40 % of lane-steps
 * are resets).  Ignored in private mode and with UCB. */
int rl_agent_set_reset_step(rl_agent *a, int32_t enable);
/* episode log (device-side reward_history / episode_length, src/agent.rs:72-141):
 * a ring of `capacity_per_lane` records per lane ([slot][lane] in HBM); 0 disables.
 * Enabling (re)allocates and empties the log. */
int rl_agent_set_episode_log(rl_agent *a, uint32_t capacity_per_lane);
/* Drain the log: records lane by lane, each lane oldest first.  n_total = records
 * available (only the first `cap` are written), n_lost = records overwritten
 * because a lane finished more than capacity_per_lane episodes.  Empties the log
 * (out == NULL only counts and keeps it). */
int rl_agent_take_episodes(rl_agent *a, rl_episode_record *out, uint64_t cap, uint64_t *n_total,
                           uint64_t *n_lost);
/* raw per-lane records (4 x u32 each): core = {s, flags|a|mode, env word, train episodes},
 * aux = {eps lo, eps hi, eval episodes left, episode length}; for checkpoints and tests */
int rl_agent_lane_state(rl_agent *a, uint32_t *core, uint32_t *aux, size_t n_lanes);

/* -------- NeuralPolicy weights (policy == RL_POLICY_NEURAL) */
/* n_in = input features, n_params = per-lane parameter count:
 * [W1 n_in x hidden][b1 hidden][W2 hidden x COUNT][b2 COUNT], row-major
 * (DenseLayer::weights is (input_size, output_size), layers.rs:61-63) */
int rl_agent_net_dims(rl_agent *a, uint32_t *n_in, uint32_t *hidden, uint32_t *n_params);
/* all lanes' parameters, [n_lanes][n_params] f64 (Layer::get_weights / get_bias) */
int rl_agent_get_weights(rl_agent *a, double *out, size_t n);
/* Layer::set_weights / set_bias for every lane, same layout */
int rl_agent_set_weights(rl_agent *a, const double *in, size_t n);
/* the input-adapter features of every dense state, [n_states][n_in] (no GPU needed) */
int rl_net_features(const rl_env_config *env, int32_t input, double *out, size_t n);

/* -------- multi-GPU (SURVEY 8(b) rl_sync, 8(e)): one process per GPU, lanes
 * partitioned contiguously (lane_offset = rank * n_lanes).  The only collectives
 * are RCCL int64 all-reduces of the merge buffer over xGMI after every launch:
 * f64 Q: a MAX over its first rl_agent_delta_max_words words (per-entry grid
 * codes), then a SUM over the rest (grid sums, group counts, ΔN, Δt, NaN/inf
 * counts); fixed point: the SUM only.  Integer sums make Q identical for any
 * rank count at a fixed global lane set.
 * Bootstrap: rank 0 calls rl_comm_unique_id and hands the bytes to every rank
 * (any channel: MPI, a file, the launcher), then each rank calls rl_comm_init. */
#define RL_COMM_ID_BYTES 128
int rl_comm_unique_id(void *id_out /* RL_COMM_ID_BYTES */);
int rl_comm_init(int32_t rank, int32_t world, const void *id /* RL_COMM_ID_BYTES */, int32_t device,
                 rl_comm **out);
void rl_comm_destroy(rl_comm *c);
int rl_comm_rank(rl_comm *c, int32_t *rank, int32_t *world);
/* host values all-reduced over the communicator's ranks, in place: op 0 = sum,
 * 1 = max, 2 = min; n == 0 is a barrier.  Blocking.  For the caller's control
 * plane (the bench's barriers and max-over-ranks time) — the merge's collectives
 * run inside the launches. */
int rl_comm_allreduce_f64(rl_comm *c, double *vals, uint32_t n, int32_t op);
/* attach (NULL: detach) a communicator: from then on every merge of rl_agent_run /
 * rl_agent_train / rl_agent_evaluate all-reduces the delta over it (train/evaluate
 * also agree on termination across ranks).  Shared mode only. */
int rl_agent_set_comm(rl_agent *a, rl_comm *c);
/* the merge of one rl_agent_launch_train: all-reduce the delta over the attached
 * communicator (none: this rank alone) on the agent's stream, then Q_base += Δ */
int rl_agent_sync(rl_agent *a);

/* -------- ABI 7: the one-shot peer-read merge
 * The merge buffers are small (cfg 2: 6 KB), so a ring all-reduce's 2(N-1) hop
 * latencies dominate it.  Instead every rank exports an exchange region by IPC;
 * a merge copies the rank's words into it, raises the rank's epoch flag
 * (system-scope release) and one kernel per rank reads all N ranks' words in rank
 * order over xGMI (int64 sums / maxima: exact, order-free) into the merge buffer.
 * rl_agent_set_comm sets this up by itself at world > 1 (the handles travel over
 * RCCL; a self-test merge agreed by every rank decides, RCCL stays on failure or
 * with RLAMD_MERGE=rccl).  Without a communicator (ranks sharing one GPU, where
 * RCCL refuses two ranks) the caller exchanges the handles:
 *   rl_agent_peer_handle on every rank -> all-gather them (rank order) ->
 *   rl_agent_peer_attach on every rank; then rl_agent_run / train / evaluate /
 *   rl_agent_sync merge over the peers.  Every rank must make the same merges, and
 *   destroy its agent only after every rank's last merge is complete (a barrier
 *   after rl_agent_synchronize): a peer may still be reading its region. */
#define RL_PEER_HANDLE_BYTES 64
int rl_agent_peer_handle(rl_agent *a, void *handle_out /* RL_PEER_HANDLE_BYTES */);
int rl_agent_peer_attach(rl_agent *a, int32_t rank, int32_t world,
                         const void *handles /* world x RL_PEER_HANDLE_BYTES, rank order */);
/* how this agent's merges are reduced: 0 this rank alone, 1 RCCL all-reduce,
 * 2 peer-read (above) */
enum rl_merge_path { RL_MERGE_LOCAL = 0, RL_MERGE_RCCL = 1, RL_MERGE_PEER = 2 };
int rl_agent_merge_path(rl_agent *a, int32_t *path);
/* ABI 7: private mode, the lanes [lane0, lane0 + n_lanes) only — Q in
 * rl_agent_get_q's [lane][P][S][A] (NeuralPolicy: get_values, [lane][S][A]) and
 * the network parameters in rl_agent_get_weights' [lane][n_params] */
int rl_agent_get_q_lanes(rl_agent *a, uint32_t lane0, uint32_t n_lanes, double *out, size_t n);
int rl_agent_get_weights_lanes(rl_agent *a, uint32_t lane0, uint32_t n_lanes, double *out, size_t n);
/* ABI 7: live eligibility-trace entries over every lane (the visited pairs of the
 * shared pair layout, visited states otherwise); 0 without traces */
int rl_agent_trace_items(rl_agent *a, uint64_t *items);

/* -------- multi-GPU: the merge as an external collective (shared mode) */
/* int64 words of the merge buffer the current Q representation uses (all of it)
 * and of its leading MAX part: f64 MAX [E] + SUM [E sums][E counts][S*A dN][1 dt]
 * [3 x E non-finite kind counts], E = the learner group's LDS entries (Blackjack
 * eps-greedy: its 2 x 484 x 2 non-terminal entries, not the 8192 dense ones); the
 * fixed point has no MAX words and SUM [PSA dQ][PSA counts][S*A dN][1 dt].  The
 * sizes change with the representation (rl_agent_q_repr): a caller-owned buffer
 * must hold the current one (a launch fails with RL_E_STATE otherwise). */
int rl_agent_delta_words(rl_agent *a, uint64_t *n);
int rl_agent_delta_max_words(rl_agent *a, uint64_t *n);
/* ABI 6: the words of the largest layout either representation can need — size a
 * caller-owned buffer by this and it survives every representation switch */
int rl_agent_delta_cap_words(rl_agent *a, uint64_t *n);
/* use caller-owned device memory (e.g. a torch int64 tensor, zeroed) as the buffer */
int rl_agent_set_delta_buffer(rl_agent *a, void *device_ptr, uint64_t n_words);
/* learner groups over every rank (the f64 merge grid's headroom; the attached
 * communicator sets it, external collectives must call this before
 * rl_agent_launch_fold: RL_E_STATE otherwise); 0 = this rank's */
int rl_agent_set_merge_groups(rl_agent *a, uint64_t total_groups);
/* one launch = train kernel (this device's part of the buffer) ...
 * [caller all-reduces the MAX words with MAX] ... */
int rl_agent_launch_train(rl_agent *a);
/* ... the grid sums (f64; nothing for the fixed point) ... [caller all-reduces the
 * remaining words with SUM] ... */
int rl_agent_launch_fold(rl_agent *a);
/* ... then Q_base = the merged values, buffer zeroed */
int rl_agent_launch_apply(rl_agent *a);
/* run on a caller stream (hipStream_t as void*); NULL = the handle's own stream */
int rl_agent_set_stream(rl_agent *a, void *stream);
/* resident train-kernel workgroups per CU (learner groups in shared mode), the
 * LDS bytes of one and its block size, for the kernel the next launch picks */
int rl_agent_occupancy(rl_agent *a, uint32_t *groups_per_cu, uint64_t *lds_bytes, uint32_t *block_threads);
/* HIP-event timing of every train kernel launch */
int rl_agent_set_timing(rl_agent *a, int32_t enable);
int rl_agent_get_timing(rl_agent *a, double *total_ms, uint64_t *n_launches);

/* -------- device known-answer probes (numerics parity; need a GPU) */
int rl_kat_log(int32_t device, const double *x, double *out, uint32_t n);
int rl_kat_rng(int32_t device, uint64_t seed, uint64_t lane, uint32_t n, uint32_t *out);
int rl_kat_ucb(int32_t device, const double *q, const double *n_count, const uint64_t *t,
               double c, double *out, uint32_t n);
/* activation f(x) and f'(x) on the device (src/network/activation.rs); act may
 * not be RL_ACT_SOFTMAX (a layer-wide function, covered by the training tests) */
int rl_kat_act(int32_t device, int32_t act, const double *x, double *f, double *fprime, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif

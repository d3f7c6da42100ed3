// rl_misc.hip — the small kernels around the fused step kernel: lane init
// (BlackJackEnv::new's deal included), train()/evaluate() arming, the group
// merge apply, the batched Env trait kernels and device KAT probes.
#include "rl_train_impl.h"

namespace rlamd {

train_launch_fn train_table_frozen_lake(int, int, int, int, int);
train_launch_fn train_table_cliff_walking(int, int, int, int, int);
train_launch_fn train_table_taxi(int, int, int, int, int);
train_launch_fn train_table_blackjack(int, int, int, int, int);
train_launch_fn train_table_frozen_lake_edited(int, int, int, int, int);

train_launch_fn lookup_train(int env, int agent, int policy, int sel, int algo, int priv) {
    switch (env) {
    case RL_ENV_FROZEN_LAKE: return train_table_frozen_lake(agent, policy, sel, algo, priv);
    case RL_ENV_CLIFF_WALKING: return train_table_cliff_walking(agent, policy, sel, algo, priv);
    case RL_ENV_TAXI: return train_table_taxi(agent, policy, sel, algo, priv);
    case RL_ENV_BLACKJACK: return train_table_blackjack(agent, policy, sel, algo, priv);
    case RL_ENV_FROZEN_LAKE_EDITED: return train_table_frozen_lake_edited(agent, policy, sel, algo, priv);
    }
    return nullptr;
}
size_t private_smem_bytes(int env, int agent, int policy, int sel, uint32_t S, uint32_t A, uint32_t n_start) {
    return smem_layout(env, policy == RL_POLICY_DOUBLE ? 2 : 1, sel == RL_SEL_UCB, agent == RL_AGENT_TRACES, S,
                       A, n_start, 0u).total;
}
size_t shared_smem_bytes(int env, int agent, int policy, int sel, int algo, uint32_t S, uint32_t A,
                         uint32_t n_start, uint32_t nthr, uint32_t trc_kb, int fq, int ucb_pack) {
    const int traces = agent != RL_AGENT_TRACES ? 0 : layout_sparse_traces(agent, sel, algo, 0) ? 2 : 1;
    const int ucb = sel != RL_SEL_UCB ? 0 : algo == RL_ALGO_EXPECTED_SARSA ? 2 : 1;
    const int P = policy == RL_POLICY_DOUBLE ? 2 : 1;
    return smem_layout(env, P, ucb, traces, S, A, n_start, nthr, trc_kb, fq, ucb_pack,
                       qsh_layout(fq, ucb, P, algo) ? 1 : 0).total;
}
uint32_t shared_pair_cap(int env, int agent, int policy, int sel, int algo, uint32_t S, uint32_t A,
                         uint32_t n_start, uint32_t nthr, uint32_t trc_kb, int fq, int ucb_pack) {
    const int traces = agent != RL_AGENT_TRACES ? 0 : layout_sparse_traces(agent, sel, algo, 0) ? 2 : 1;
    const int ucb = sel != RL_SEL_UCB ? 0 : algo == RL_ALGO_EXPECTED_SARSA ? 2 : 1;
    const int P = policy == RL_POLICY_DOUBLE ? 2 : 1;
    return smem_layout(env, P, ucb, traces, S, A, n_start, nthr, trc_kb, fq, ucb_pack,
                       qsh_layout(fq, ucb, P, algo) ? 1 : 0).trc_cap;
}
// the envs whose shared pair lists append through pair_visit (slot_of + vbits for
// the HBM slots); the small tables keep their pair bits in registers (PBITS in
// train_shared_body) and never read either
bool pair_slot_index_env(int env) {
    return !(RLAMD_COOP_SWEEP && RLAMD_PAIR_BITS &&
             (env == RL_ENV_CLIFF_WALKING || env == RL_ENV_FROZEN_LAKE || env == RL_ENV_FROZEN_LAKE_EDITED));
}

// ---------------------------------------------------------------- pair-trace re-index
// A lane's pair list keeps slots [0, cap) in LDS during a launch and [cap, np) in
// HBM with slot_of[id] and the visited-state bitmap vbits covering the HBM part
// only (pair_visit).  Positions and first-of-state flags do not depend on cap, so
// when a launch runs with another cap than the last (the carve of the
// other kernel family, or a selector switch) the index of its HBM part is rebuilt
// here: vbits cleared (a grown cap leaves bits of slots now in LDS, which the
// episode end would no longer clear), then slot_of / vbits for [cap, np).
__global__ void k_pair_reindex(KParams p, uint32_t cap) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= p.L) return;
    const uint64_t Ls = p.L;
    const uint32_t np = p.tcnt[lane], nw = (p.S + 31u) >> 5;
    for (uint32_t w = 0; w < nw; ++w) p.vbits[(uint64_t)w * Ls + lane] = 0u;
    for (uint32_t j = cap; j < np; ++j) {
        const uint32_t id = p.tlist[pslot(p, j, lane)] & 0x7fffu, s = id / p.A;
        p.slot_of[(uint64_t)id * Ls + lane] = (uint16_t)j;
        uint32_t *vw = &p.vbits[(uint64_t)(s >> 5) * Ls + lane];
        *vw = *vw | (1u << (s & 31u));
    }
}
void launch_pair_reindex(const KParams &p, uint32_t cap, hipStream_t s) {
    hipLaunchKernelGGL(k_pair_reindex, dim3((unsigned)((p.L + 255) / 256)), dim3(256), 0, s, p, cap);
}

// ---------------------------------------------------------------- lane init
// Fresh lanes: RNG keyed (seed, global lane), need_reset, DoubleTabularPolicy
// flag = true, epsilon = eps0.  Blackjack consumes BlackJackEnv::new()'s deal
// (blackjack.rs:32-46) so the stream matches a freshly constructed reference env.
__global__ void k_lane_init(KParams p, int env, uint64_t seed, uint64_t lane_offset, double eps0) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= p.L) return;
    const uint4 r0 = rng_seed(seed, lane_offset + lane);
    Rng r{r0.x, r0.y, r0.z, r0.w};
    uint32_t z = 0;
    if (env == RL_ENV_BLACKJACK) z = EnvDev<RL_ENV_BLACKJACK>::deal(r);
    p.core[lane] = make_uint4(0, LF_NEED_RESET | LF_DFLAG | ((uint32_t)RL_MODE_TRAIN << LF_MODE_SHIFT), z, 0);
    p.rng[lane] = make_uint4(r.s0, r.s1, r.s2, r.s3);
    const uint64_t e = (uint64_t)__double_as_longlong(eps0);
    p.aux[lane] = make_uint4((uint32_t)e, (uint32_t)(e >> 32), 0, 0);
    p.epi_reward[lane] = 0.0;
}
void launch_lane_init(int env, const KParams &p, uint64_t seed, uint64_t lane_offset, double eps0,
                      hipStream_t s) {
    hipLaunchKernelGGL(k_lane_init, dim3((p.L + 255) / 256), dim3(256), 0, s, p, env, seed, lane_offset, eps0);
}

// ---------------------------------------------------------------- arm
// start of Agent::train / Agent::evaluate: every lane begins a new episode
// (src/agent.rs:83 env.reset()), episode counter 0, mode set.  mode < 0 keeps
// the mode and only restores epsilon (Agent::reset / set_action_selector).
__global__ void k_arm(KParams p, int32_t mode, uint32_t eval_left, int restore_eps, double eps0) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= p.L) return;
    uint4 c = p.core[lane];
    uint4 x = p.aux[lane];
    if (mode >= 0) {
        c.y = (c.y & (LF_ACT_MASK | LF_READY | LF_DFLAG)) | LF_NEED_RESET | ((uint32_t)mode << LF_MODE_SHIFT);
        c.w = 0;
        x.z = eval_left;
    }
    if (restore_eps) {
        const uint64_t e = (uint64_t)__double_as_longlong(eps0);
        x.x = (uint32_t)e; x.y = (uint32_t)(e >> 32);
    }
    p.core[lane] = c;
    p.aux[lane] = x;
}
void launch_arm_full(const KParams &p, int32_t mode, uint32_t eval_left, int restore_eps, double eps0,
                     hipStream_t s) {
    hipLaunchKernelGGL(k_arm, dim3((p.L + 255) / 256), dim3(256), 0, s, p, mode, eval_left, restore_eps, eps0);
}

__global__ void k_fill_f64(double *ptr, uint64_t n, double v) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ptr[i] = v;
}
void launch_fill_f64(double *ptr, uint64_t n, double v, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_fill_f64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ptr, n, v);
}

// ---------------------------------------------------------------- loop control word
// train()/evaluate()'s exit agreement, formed on the device after each launch:
// ctl = {lanes DONE (stats slot 5 over the replicas), lanes, status}; the caller
// sums it over the ranks (one 24-byte all-reduce) and reads it one launch later.
__global__ void __launch_bounds__(64) k_ctl_word(const unsigned long long *stats, int64_t *ctl, uint64_t lanes,
                                                 int64_t status) {
    const uint32_t t = threadIdx.x;
    uint64_t v = 0;
    for (uint32_t r = t; r < STATS_REP; r += 64u) v += stats[(uint64_t)r * STATS_W + 5u];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (t == 0) {
        ctl[0] = (int64_t)v;
        ctl[1] = (int64_t)lanes;
        ctl[2] = status;
    }
}
void launch_ctl_word(const KParams &p, int64_t *ctl, uint64_t lanes, int64_t status, hipStream_t s) {
    hipLaunchKernelGGL(k_ctl_word, dim3(1), dim3(64), 0, s, p.stats, ctl, lanes, status);
}

// ---------------------------------------------------------------- peer-read merge
// the all-reduce of a small merge buffer as one read of every rank's
// words over xGMI.  Each rank's exchange region (uncached device memory, exported
// by IPC; rl_host.cpp PeerMerge) holds two slots of `cap` words and, 128 B past
// them, the rank's epoch flag.  Merge e (1, 2, ...) uses slot e & 1:
//   k_peer_put     the rank's words -> its own slot (system-scope stores: they
//                  reach memory, not a cache another GPU cannot see);
//   k_peer_reduce  block 0 raises the rank's flag to e (system-scope release),
//                  every block waits until each peer's flag is >= e (system-scope
//                  acquire, bounded), then sums (or takes the max of) the N
//                  ranks' words in rank order into the merge buffer — int64, so
//                  exact and order-free.
// Slot reuse is safe with two slots: a rank rewrites slot e & 1 at merge e + 2
// only after its merge e + 1 saw every peer's flag at e + 1, which a peer raises
// only after its own reads of merge e are done (same stream, in order).
// A peer that never arrives (a crashed rank) ends the wait after timeout_ticks of
// the wall clock with *err set, so no kernel spins forever.
__global__ void k_peer_put(const int64_t *src, int64_t *slot, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) __hip_atomic_store(&slot[i], src[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// block 0 raises this rank's flag to `epoch`; every block waits until each peer's
// flag is >= epoch (or the wall clock passes timeout_ticks: *err set).  Every
// thread of the block calls it (one barrier); true when the peers arrived
__device__ __forceinline__ bool peer_arrive_wait(int64_t *const *bases, uint32_t world, uint32_t rank,
                                                 uint64_t flag_off, int64_t epoch, uint32_t *err,
                                                 int64_t timeout_ticks) {
    __shared__ uint32_t timed_out;
    if (threadIdx.x == 0) {
        timed_out = 0u;
        if (blockIdx.x == 0)
            __hip_atomic_store(&bases[rank][flag_off], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        const int64_t t0 = wall_clock64();
        for (uint32_t r = 0; r < world && !timed_out; ++r) {
            if (r == rank) continue;
            while (__hip_atomic_load(&bases[r][flag_off], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
                __builtin_amdgcn_s_sleep(2);
                if (wall_clock64() - t0 > timeout_ticks) {
                    timed_out = 1u;
                    atomicOr(err, 1u);
                    break;
                }
            }
        }
    }
    __syncthreads();
    return timed_out == 0u;
}
__global__ void __launch_bounds__(256) k_peer_reduce(int64_t *const *bases, uint32_t world, uint32_t rank,
                                                     uint64_t slot_off, uint64_t flag_off, uint64_t n,
                                                     int64_t epoch, int32_t op_max, int64_t *dst, uint32_t *err,
                                                     int64_t timeout_ticks) {
    const bool ok = peer_arrive_wait(bases, world, rank, flag_off, epoch, err, timeout_ticks);
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (!ok || i >= n) return;
    int64_t acc = op_max ? INT64_MIN : 0;
    for (uint32_t r = 0; r < world; ++r) {
        const int64_t v = __hip_atomic_load(&bases[r][slot_off + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        acc = op_max ? (v > acc ? v : acc) : (int64_t)((uint64_t)acc + (uint64_t)v);
    }
    dst[i] = acc;
}
void launch_peer_put(const int64_t *src, int64_t *slot, uint64_t n, hipStream_t s) {
    if (n) hipLaunchKernelGGL(k_peer_put, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, slot, n);
}
void launch_peer_reduce(int64_t *const *bases, uint32_t world, uint32_t rank, uint64_t slot_off, uint64_t flag_off,
                        uint64_t n, int64_t epoch, int op_max, int64_t *dst, uint32_t *err, int64_t timeout_ticks,
                        hipStream_t s) {
    // at least one block: block 0 raises the flag even for n == 0
    hipLaunchKernelGGL(k_peer_reduce, dim3((unsigned)(n ? (n + 255) / 256 : 1)), dim3(256), 0, s,
                       bases, world, rank, slot_off, flag_off, n, epoch, op_max, dst, err, timeout_ticks);
}

// The fixed-point merge over the peers in two launches instead of four (round 6):
// the replicas folded straight into this rank's exchange slot (k_peer_fold_put:
// k_fold_replicas' sum written with system-scope stores), then the N ranks' words
// reduced and applied in one pass (k_peer_reduce_apply: k_apply's rule on the
// rank-order sums — Q_base += mean_delta(Σ dQ, Σ counts), N / t += Σ Δ).
__global__ void __launch_bounds__(256) k_peer_fold_put(KParams p, int64_t *slot) {
    __shared__ uint64_t part[4][64];
    const uint32_t lw = threadIdx.x & 63u, g = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * 64u + lw;
    uint64_t s = 0;
    if (w < p.sum_words) {
        int64_t *x = p.delta_rep + (uint64_t)g * p.delta_words + w;
        const uint64_t stride = 4ull * p.delta_words;
        const uint32_t n = p.n_rep > g ? (p.n_rep - g + 3u) / 4u : 0u;
#pragma unroll 16
        for (uint32_t i = 0; i < n; ++i) s += (uint64_t)x[i * stride];
#pragma unroll 16
        for (uint32_t i = 0; i < n; ++i) x[i * stride] = 0;
    }
    part[g][lw] = s;
    __syncthreads();
    if (g == 0 && w < p.sum_words) {
        const int64_t v = (int64_t)((uint64_t)p.delta[w] + part[0][lw] + part[1][lw] + part[2][lw] + part[3][lw]);
        __hip_atomic_store(&slot[w], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        p.delta[w] = 0;
    }
}
__global__ void __launch_bounds__(256) k_peer_reduce_apply(KParams p, int64_t *const *bases, uint32_t world,
                                                           uint32_t rank, uint64_t slot_off, uint64_t flag_off,
                                                           int64_t epoch, uint32_t *err, int64_t timeout_ticks) {
    const bool ok = peer_arrive_wait(bases, world, rank, flag_off, epoch, err, timeout_ticks);
    const uint32_t PSA = p.P * p.S * p.A, SA = p.S * p.A;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (!ok) return;
    auto rsum = [&](uint64_t w) -> int64_t {   // the ranks' words in rank order (exact)
        uint64_t acc = 0;
        for (uint32_t r = 0; r < world; ++r)
            acc += (uint64_t)__hip_atomic_load(&bases[r][slot_off + w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return (int64_t)acc;
    };
    if (i < PSA) p.q_base[i] = p.q_base[i] + mean_delta(rsum(i), rsum(PSA + i));
    if (i < SA) p.n_base[i] = p.n_base[i] + (uint64_t)rsum(2ull * PSA + i);
    if (i == 0) p.t_base[0] = (uint64_t)((int64_t)p.t_base[0] + rsum(2ull * PSA + SA));
}
void launch_peer_fold_put(const KParams &p, int64_t *slot, hipStream_t s) {
    hipLaunchKernelGGL(k_peer_fold_put, dim3((p.sum_words + 63) / 64), dim3(256), 0, s, p, slot);
}
void launch_peer_reduce_apply(const KParams &p, int64_t *const *bases, uint32_t world, uint32_t rank,
                              uint64_t slot_off, uint64_t flag_off, int64_t epoch, uint32_t *err,
                              int64_t timeout_ticks, hipStream_t s) {
    const uint32_t PSA = p.P * p.S * p.A;
    hipLaunchKernelGGL(k_peer_reduce_apply, dim3((PSA + 255) / 256), dim3(256), 0, s, p, bases, world, rank,
                       slot_off, flag_off, epoch, err, timeout_ticks);
}

// ---------------------------------------------------------------- replica fold
// delta += sum over replicas (exact int64), replicas zeroed for the next launch.
// Block = 64 words x 4 replica slices; each thread's replica loads are
// independent (unrolled) so they are in flight together.
__global__ void __launch_bounds__(256) k_fold_replicas(KParams p) {
    __shared__ uint64_t part[4][64];
    const uint32_t lw = threadIdx.x & 63u, g = threadIdx.x >> 6;
    const uint64_t w = (uint64_t)blockIdx.x * 64u + lw;
    uint64_t s = 0;
    if (w < p.sum_words) {
        int64_t *x = p.delta_rep + (uint64_t)g * p.delta_words + w;
        const uint64_t stride = 4ull * p.delta_words;
        const uint32_t n = p.n_rep > g ? (p.n_rep - g + 3u) / 4u : 0u;
#pragma unroll 16
        for (uint32_t i = 0; i < n; ++i) s += (uint64_t)x[i * stride];
#pragma unroll 16
        for (uint32_t i = 0; i < n; ++i) x[i * stride] = 0;
    }
    part[g][lw] = s;
    __syncthreads();
    if (g == 0 && w < p.sum_words)
        p.delta[w] = (int64_t)((uint64_t)p.delta[w] + part[0][lw] + part[1][lw] + part[2][lw] + part[3][lw]);
}
void launch_fold_replicas(const KParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_fold_replicas, dim3((p.sum_words + 63) / 64), dim3(256), 0, s, p);
}

// ---------------------------------------------------------------- fused fold + apply
// One-process merge of an eps-greedy learner in the fixed point (the delta holds
// [PSA sums][PSA counts] only: no UCB counters): entry i sums its two words over
// the replicas (4 replica slices per block, as k_fold_replicas), zeroes them and
// applies k_apply's rule, Q_base[i] += mean (in range: the host's proof).  One
// launch instead of two.
__global__ void __launch_bounds__(256) k_fold_apply(KParams p) {
    __shared__ uint64_t part[2][4][64];
    const uint32_t PSA = p.P * p.S * p.A;
    const uint32_t lw = threadIdx.x & 63u, g = threadIdx.x >> 6;
    const uint32_t i = blockIdx.x * 64u + lw;
    uint64_t s = 0, c = 0;
    if (i < PSA) {
        int64_t *x = p.delta_rep + (uint64_t)g * p.delta_words + i;
        const uint64_t stride = 4ull * p.delta_words;
        const uint32_t n = p.n_rep > g ? (p.n_rep - g + 3u) / 4u : 0u;
#pragma unroll 8
        for (uint32_t r = 0; r < n; ++r) {
            s += (uint64_t)x[r * stride];
            c += (uint64_t)x[r * stride + PSA];
        }
#pragma unroll 8
        for (uint32_t r = 0; r < n; ++r) {
            x[r * stride] = 0;
            x[r * stride + PSA] = 0;
        }
    }
    part[0][g][lw] = s;
    part[1][g][lw] = c;
    __syncthreads();
    if (g == 0 && i < PSA) {
        int64_t *d = p.delta;
        const int64_t sum = (int64_t)((uint64_t)d[i] + part[0][0][lw] + part[0][1][lw] + part[0][2][lw] + part[0][3][lw]);
        const int64_t cnt = (int64_t)((uint64_t)d[PSA + i] + part[1][0][lw] + part[1][1][lw] + part[1][2][lw] +
                                      part[1][3][lw]);
        p.q_base[i] = p.q_base[i] + mean_delta(sum, cnt);
        d[i] = 0;
        d[PSA + i] = 0;
    }
}
void launch_fold_apply(const KParams &p, hipStream_t s) {
    const uint32_t PSA = p.P * p.S * p.A;
    hipLaunchKernelGGL(k_fold_apply, dim3((PSA + 63) / 64), dim3(256), 0, s, p);
}

// ---------------------------------------------------------------- merge apply
// Fixed point: Q_base += mean of the groups' (and ranks') ΔQ, already summed by
// global int64 atomics and, across GPUs, by the caller's all-reduce.  Both
// representations: UCB counters summed.  Then Δ = 0 for the next launch.
__global__ void k_apply(KParams p) {
    const uint32_t PSA = p.P * p.S * p.A, SA = p.S * p.A;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    int64_t *d = p.delta;
    if (i < PSA && !p.fq) {   // Q_base += mean over the groups (and ranks) that changed the entry
        p.q_base[i] = p.q_base[i] + mean_delta(d[i], d[PSA + i]);
        d[i] = 0;
        d[PSA + i] = 0;
    }
    if (i < SA) {    // UCB counters are counts: summed
        p.n_base[i] = p.n_base[i] + (uint64_t)d[2 * PSA + i];
        d[2 * PSA + i] = 0;
    }
    if (i == 0) {
        p.t_base[0] = (uint64_t)((int64_t)p.t_base[0] + d[2 * PSA + SA]);
        d[2 * PSA + SA] = 0;
    }
}
void launch_apply(const KParams &p, hipStream_t s) {
    const uint32_t PSA = p.P * p.S * p.A;
    hipLaunchKernelGGL(k_apply, dim3((PSA + 255) / 256), dim3(256), 0, s, p);
}

// ---------------------------------------------------------------- f64 merge
// Every group left its final Q (LDS order) in qslot[group][psal].  An entry that
// some groups changed (bits differ from Q_base) takes the MEAN of their values
// (oracle rlref.c rlo_batch_launch_groups / _fold / _apply_delta):
//   a: per entry the max code over the changed finite values (MAX words), the
//      number of changed groups and of NaN / +inf / -inf values (SUM words);
//   b: the changed finite values on the grid 2^(max(code,1) - 1075 + merge_hb),
//      summed (exact int64; merge_hb keeps 2^(10+hb) groups below 2^63);
//   apply: Q_base = IEEE kind if any non-finite, else ldexp(fl(sum * fl(1/n)), e).
// Across ranks: MAX all-reduce between a and b, SUM all-reduce between b and apply.
// Grid: (entry blocks of 64) x (group blocks of 64); 256 threads = 64 entries x
// 4 group slices of 16 groups.
// The merge buffer is indexed by the LDS entry j (psal entries: Blackjack
// eps-greedy holds only its 484 non-terminal rows, the only ones an update can
// write), so the MAX words are [psal] and the SUM words [psal sums][psal counts]
// [SA dN][1 dt][3 x psal kind counts]: cfg 5's all-reduced merge is 5x smaller
// than over the 2048 dense rows.  UCB keeps dense rows (psal == P*S*A).
__device__ __forceinline__ uint32_t fq_dense(const KParams &p, uint32_t j) {   // LDS index -> dense [P][S][A]
    if (p.psal == p.P * p.S * p.A) return j;
    const uint32_t A = p.A, SAL = BJ_LDS_STATES * A, tbl = j / SAL, r = j - tbl * SAL;
    return tbl * p.S * A + bj_dense(r / A) * A + r % A;
}
__global__ void __launch_bounds__(256) k_fq_merge_a(KParams p) {
    __shared__ uint32_t code[4][64], cnt[4][64], kinds[3][4][64];
    const uint32_t lw = threadIdx.x & 63u, gs = threadIdx.x >> 6;
    const uint32_t j = blockIdx.x * 64u + lw;
    uint32_t c = 0, n = 0, kn = 0, kp = 0, km = 0;
    if (j < p.psal) {
        const uint32_t i = fq_dense(p, j);
        const uint64_t base = (uint64_t)p.q_base[i];
        const uint32_t g0 = blockIdx.y * 64u + gs * 16u;
#pragma unroll 4
        for (uint32_t g = g0; g < g0 + 16u && g < p.n_groups; ++g) {
            const uint64_t v = p.qslot[(uint64_t)g * p.psal + j];
            if (v == base) continue;
            ++n;
            const double x = as_f64(v);
            if (__builtin_isfinite(x)) {
                const uint32_t cd = f64_code(x);
                c = cd > c ? cd : c;
            } else {
                const uint32_t f = nf_flag(x);
                kn += f == QF_NAN;
                kp += f == QF_PINF;
                km += f == QF_NINF;
            }
        }
    }
    code[gs][lw] = c; cnt[gs][lw] = n; kinds[0][gs][lw] = kn; kinds[1][gs][lw] = kp; kinds[2][gs][lw] = km;
    __syncthreads();
    if (gs == 0 && j < p.psal) {
        const uint32_t PS = p.psal;
        uint32_t cm = 0, nt = 0, k0 = 0, k1 = 0, k2 = 0;
        for (int q = 0; q < 4; ++q) {
            cm = code[q][lw] > cm ? code[q][lw] : cm;
            nt += cnt[q][lw]; k0 += kinds[0][q][lw]; k1 += kinds[1][q][lw]; k2 += kinds[2][q][lw];
        }
        if (cm) atomicMax((unsigned long long *)&p.delta_max[j], (unsigned long long)cm);
        int64_t *d = p.delta, *fc = d + 2 * PS + p.S * p.A + 1;
        if (nt) atomicAdd((unsigned long long *)&d[PS + j], (unsigned long long)nt);
        if (k0) atomicAdd((unsigned long long *)&fc[j], (unsigned long long)k0);
        if (k1) atomicAdd((unsigned long long *)&fc[PS + j], (unsigned long long)k1);
        if (k2) atomicAdd((unsigned long long *)&fc[2 * PS + j], (unsigned long long)k2);
    }
}
__global__ void __launch_bounds__(256) k_fq_merge_b(KParams p) {
    __shared__ int64_t part[4][64];
    const uint32_t lw = threadIdx.x & 63u, gs = threadIdx.x >> 6;
    const uint32_t j = blockIdx.x * 64u + lw;
    int64_t sum = 0;
    if (j < p.psal) {
        const uint64_t base = (uint64_t)p.q_base[fq_dense(p, j)];
        const int e = fq_grid((uint32_t)p.delta_max[j]) + p.merge_hb;
        const uint32_t g0 = blockIdx.y * 64u + gs * 16u;
#pragma unroll 4
        for (uint32_t g = g0; g < g0 + 16u && g < p.n_groups; ++g) {
            const uint64_t v = p.qslot[(uint64_t)g * p.psal + j];
            const double x = as_f64(v);
            if (v != base && __builtin_isfinite(x)) sum += fq_raw(x, e);
        }
    }
    part[gs][lw] = sum;
    __syncthreads();
    if (gs == 0 && j < p.psal) {
        const int64_t t = part[0][lw] + part[1][lw] + part[2][lw] + part[3][lw];
        if (t) atomicAdd((unsigned long long *)&p.delta[j], (unsigned long long)t);
    }
}
// Q_base = the merged value of every entry some group changed.  The grid sums are
// exact only while the changed groups (over every rank) number at most
// 2^(10 + merge_hb) (rl_host.cpp merge_headroom); a larger count — an external
// collective over more groups than rl_agent_set_merge_groups declared — is counted
// in rl_stats.delta_saturations, and train / evaluate fail on it.
__global__ void k_fq_apply(KParams p) {
    const uint32_t PS = p.psal, SA = p.S * p.A;
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    int64_t *d = p.delta, *fc = d + 2 * PS + SA + 1;
    if (j < PS) {
        const uint64_t n = (uint64_t)d[PS + j];
        if (n) {
            const uint32_t f = (fc[j] ? QF_NAN : 0u) | (fc[PS + j] ? QF_PINF : 0u) | (fc[2 * PS + j] ? QF_NINF : 0u);
            double v;
            if (f) v = nf_value(f);
            else v = __builtin_ldexp((double)d[j] * (1.0 / (double)n), fq_grid((uint32_t)p.delta_max[j]) + p.merge_hb);
            p.q_base[fq_dense(p, j)] = (int64_t)f64_bits(canon_nan(v));
            if (n > (1ull << (10 + p.merge_hb)))
                atomicAdd(&p.stats[(blockIdx.x % STATS_REP) * STATS_W + ACC_SAT], 1ull);
        }
        d[j] = 0;
        d[PS + j] = 0;
        fc[j] = fc[PS + j] = fc[2 * PS + j] = 0;
        p.delta_max[j] = 0;
    }
    if (j < SA) {
        p.n_base[j] = p.n_base[j] + (uint64_t)d[2 * PS + j];
        d[2 * PS + j] = 0;
    }
    if (j == 0) {
        p.t_base[0] = (uint64_t)((int64_t)p.t_base[0] + d[2 * PS + SA]);
        d[2 * PS + SA] = 0;
    }
}
void launch_fq_merge_a(const KParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_fq_merge_a, dim3((p.psal + 63) / 64, (p.n_groups + 63) / 64), dim3(256), 0, s, p);
}
void launch_fq_merge_b(const KParams &p, hipStream_t s) {
    hipLaunchKernelGGL(k_fq_merge_b, dim3((p.psal + 63) / 64, (p.n_groups + 63) / 64), dim3(256), 0, s, p);
}
void launch_fq_apply(const KParams &p, hipStream_t s) {
    const uint32_t n = p.psal > p.S * p.A ? p.psal : p.S * p.A;
    hipLaunchKernelGGL(k_fq_apply, dim3((n + 255) / 256), dim3(256), 0, s, p);
}

// ---------------------------------------------------------------- batched Env trait
template <int ENV>
__global__ void k_env_reset(KParams p, uint64_t *obs) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= p.L) return;
    EnvTables t{p.trans, p.start_cdf, p.n_start, p.max_steps, p.th1, p.th2, p.th3, p.trunc_reward,
                p.fixed_start, p.slippery, p.S};
    uint4 c = p.core[lane];
    const uint4 r0 = p.rng[lane];
    Rng r{r0.x, r0.y, r0.z, r0.w};
    c.x = EnvDev<ENV>::reset(c.z, r, t);
    c.y |= LF_READY;
    p.core[lane] = c;
    p.rng[lane] = make_uint4(r.s0, r.s1, r.s2, r.s3);
    obs[lane] = c.x;
}
template <int ENV>
__global__ void k_env_step(KParams p, const uint32_t *act, uint64_t *obs, double *rew, uint8_t *term) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= p.L) return;
    EnvTables t{p.trans, p.start_cdf, p.n_start, p.max_steps, p.th1, p.th2, p.th3, p.trunc_reward,
                p.fixed_start, p.slippery, p.S};
    uint4 c = p.core[lane];
    const uint4 r0 = p.rng[lane];
    Rng r{r0.x, r0.y, r0.z, r0.w};
    uint32_t s2 = 0;
    double rw = 0.0;
    bool tm = false;
    uint32_t pos = c.x;
    EnvDev<ENV>::step(pos, c.z, act[lane], r, t, s2, rw, tm);
    c.x = s2;
    if (tm) c.y &= ~LF_READY;
    p.core[lane] = c;
    p.rng[lane] = make_uint4(r.s0, r.s1, r.s2, r.s3);
    obs[lane] = s2;
    rew[lane] = rw;
    term[lane] = (uint8_t)tm;
}
void launch_env_reset(int env, const KParams &p, hipStream_t s, uint64_t *obs) {
    const dim3 g((p.L + 255) / 256), b(256);
    switch (env) {
    case RL_ENV_FROZEN_LAKE: hipLaunchKernelGGL(k_env_reset<RL_ENV_FROZEN_LAKE>, g, b, 0, s, p, obs); break;
    case RL_ENV_CLIFF_WALKING: hipLaunchKernelGGL(k_env_reset<RL_ENV_CLIFF_WALKING>, g, b, 0, s, p, obs); break;
    case RL_ENV_TAXI: hipLaunchKernelGGL(k_env_reset<RL_ENV_TAXI>, g, b, 0, s, p, obs); break;
    case RL_ENV_BLACKJACK: hipLaunchKernelGGL(k_env_reset<RL_ENV_BLACKJACK>, g, b, 0, s, p, obs); break;
    case RL_ENV_FROZEN_LAKE_EDITED: hipLaunchKernelGGL(k_env_reset<RL_ENV_FROZEN_LAKE_EDITED>, g, b, 0, s, p, obs); break;
    }
}
void launch_env_step(int env, const KParams &p, hipStream_t s, const uint32_t *act, uint64_t *obs,
                     double *rew, uint8_t *term, unsigned int *) {
    const dim3 g((p.L + 255) / 256), b(256);
    switch (env) {
    case RL_ENV_FROZEN_LAKE: hipLaunchKernelGGL(k_env_step<RL_ENV_FROZEN_LAKE>, g, b, 0, s, p, act, obs, rew, term); break;
    case RL_ENV_CLIFF_WALKING: hipLaunchKernelGGL(k_env_step<RL_ENV_CLIFF_WALKING>, g, b, 0, s, p, act, obs, rew, term); break;
    case RL_ENV_TAXI: hipLaunchKernelGGL(k_env_step<RL_ENV_TAXI>, g, b, 0, s, p, act, obs, rew, term); break;
    case RL_ENV_BLACKJACK: hipLaunchKernelGGL(k_env_step<RL_ENV_BLACKJACK>, g, b, 0, s, p, act, obs, rew, term); break;
    case RL_ENV_FROZEN_LAKE_EDITED: hipLaunchKernelGGL(k_env_step<RL_ENV_FROZEN_LAKE_EDITED>, g, b, 0, s, p, act, obs, rew, term); break;
    }
}

// ---------------------------------------------------------------- NeuralPolicy
// DenseLayer::new (gen 0) / DenseLayer::reset (gen k >= 1) of every lane's network
// (src/network/layers.rs:55-73, :90-95): W ~ rand 0.8.5 Uniform::new(-l, l) drawn
// row-major from the lane's weight stream (seed ^ 0xD1B54A32D192ED03*(gen+1),
// global lane), value0_1 * scale + low; b = 0 (new) or 0.1 (reset).  The host
// passes each layer's (scale, low) (UniformFloat::new's scale search).
__global__ void k_net_init(KParams p, uint64_t seed, uint64_t lane_offset, uint32_t gen, double scale1, double low1,
                           double scale2, double low2) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= p.L) return;
    const uint4 r0 = rng_seed(seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(gen + 1u)), lane_offset + lane);
    Rng r{r0.x, r0.y, r0.z, r0.w};
    const uint32_t nw1 = p.n_in * p.n_hidden, nw2 = p.n_hidden * p.A;
    const double bias = gen ? 0.1 : 0.0;
    uint32_t k = 0;
    for (uint32_t i = 0; i < nw1; ++i, ++k) {
        const uint64_t bits = (r.next_u64() >> 12) | 0x3FF0000000000000ull;
        p.net_w[(uint64_t)k * p.L + lane] = (__longlong_as_double((long long)bits) - 1.0) * scale1 + low1;
    }
    for (uint32_t i = 0; i < p.n_hidden; ++i, ++k) p.net_w[(uint64_t)k * p.L + lane] = bias;
    for (uint32_t i = 0; i < nw2; ++i, ++k) {
        const uint64_t bits = (r.next_u64() >> 12) | 0x3FF0000000000000ull;
        p.net_w[(uint64_t)k * p.L + lane] = (__longlong_as_double((long long)bits) - 1.0) * scale2 + low2;
    }
    for (uint32_t i = 0; i < p.A; ++i, ++k) p.net_w[(uint64_t)k * p.L + lane] = bias;
}
void launch_net_init(const KParams &p, uint64_t seed, uint64_t lane_offset, uint32_t gen, double scale1,
                     double low1, double scale2, double low2, hipStream_t s) {
    hipLaunchKernelGGL(k_net_init, dim3((p.L + 255) / 256), dim3(256), 0, s, p, seed, lane_offset, gen, scale1, low1,
                       scale2, low2);
}
// Policy::get_values of every state for every lane: out[lane][s][a]
template <int A>
__global__ void k_net_values(KParams p, double *out) {
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (lane >= p.L) return;
    const NetLane n{p.net_w, p.L, lane, p.n_in, p.n_hidden, (uint32_t)A};
    for (uint32_t st = 0; st < p.S; ++st) {
        double x[NET_MAX_IN], opre[A], y[A];
        net_input(p, st, x);
        net_forward<A>(p, n, x, opre, y);
#pragma unroll
        for (int i = 0; i < A; ++i) out[(lane * p.S + st) * A + i] = y[i];
    }
}
void launch_net_values(const KParams &p, double *out, hipStream_t s) {
    const dim3 g((p.L + 255) / 256), b(256);
    switch (p.A) {
    case 2: hipLaunchKernelGGL(k_net_values<2>, g, b, 0, s, p, out); break;
    case 4: hipLaunchKernelGGL(k_net_values<4>, g, b, 0, s, p, out); break;
    case 6: hipLaunchKernelGGL(k_net_values<6>, g, b, 0, s, p, out); break;
    }
}

// ---------------------------------------------------------------- KAT probes
__global__ void k_kat_act(int act, const double *x, double *f, double *fp, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { f[i] = act_f(act, x[i]); fp[i] = act_fp(act, x[i]); }
}
void launch_kat_act(int act, const double *x, double *f, double *fp, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_kat_act, dim3((n + 255) / 256), dim3(256), 0, s, act, x, f, fp, n);
}

__global__ void k_kat_log(const double *x, double *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rl_log(x[i]);
}
__global__ void k_kat_rng(uint64_t seed, uint64_t lane, uint32_t n, uint32_t *out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint4 r0 = rng_seed(seed, lane);
    Rng r{r0.x, r0.y, r0.z, r0.w};
    for (uint32_t i = 0; i < n; ++i) out[i] = r.next_u32();
}
__global__ void k_kat_ucb(const double *q, const double *nc, const uint64_t *t, double c, double *out,
                          uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = ucb_value(q[i], c, rl_log((double)t[i]), nc[i]);
}
void launch_kat_log(const double *x, double *out, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_kat_log, dim3((n + 255) / 256), dim3(256), 0, s, x, out, n);
}
void launch_kat_rng(uint64_t seed, uint64_t lane, uint32_t n, uint32_t *out, hipStream_t s) {
    hipLaunchKernelGGL(k_kat_rng, dim3(1), dim3(64), 0, s, seed, lane, n, out);
}
void launch_kat_ucb(const double *q, const double *nc, const uint64_t *t, double c, double *out,
                    uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_kat_ucb, dim3((n + 255) / 256), dim3(256), 0, s, q, nc, t, c, out, n);
}

}  // namespace rlamd

// rl_train_impl.h — the fused training-step kernels (included by rl_train_<env>.hip).
//
// One thread = one env lane.  A launch runs K = sync_every synchronous steps of
// Agent::train's loop body (src/agent.rs:86-106) for every lane, entirely in
// registers / LDS; lane records are read once and written once per launch.
//
//  k_train_shared : a workgroup is a learner group of G lanes sharing one Q
//                   copy in LDS as int64 fixed point (2^-40).  Each step: reads
//                   against the step-start snapshot, then every lane's delta is
//                   added with ds_add_u64 (integer: order free, bit-reproducible),
//                   then the group's ΔQ goes to HBM by global int64 atomics.
//  k_train_private: group_size == 1.  Every lane is a complete reference agent
//                   with f64 Q / UCB counters in HBM (SoA [entry][lane]) — the
//                   reference's arithmetic bit for bit.
#pragma once
#include <type_traits>

#include "rl_device.h"
#include "rl_net.h"

namespace rlamd {

#ifndef RLAMD_FUSE_MAX
#define RLAMD_FUSE_MAX 2   // single-table Q-learning: one argmax+max pass per step (0: off,
                           // 1: fused, 2: fused and pinned before the selection)
#endif

// Pair pools (the small-table traces kernel, cfg 4):
//  RLAMD_POOL_BF    the item body branch-free: every item of a round adds its
//                   contribution and its row count (0 for the items of lanes that
//                   do not train), the non-finite case behind one wave-uniform test,
//                   the keep-write's LDS / HBM choice uniform while the round fits
//  RLAMD_POOL_REC16 an item's tag and E as one 16-byte LDS record (one ds_read_b128
//                   and one ds_write_b128 per item instead of a u16 and an f64 each)
//  RLAMD_POOL_LREC  each lane's {td, pk} in a 16-byte LDS record read by its items
//                   (one ds_read_b128) instead of three ds_bpermute
#ifndef RLAMD_POOL_BF
#define RLAMD_POOL_BF 0
#endif
#ifndef RLAMD_POOL_REC16
#define RLAMD_POOL_REC16 0
#endif
#ifndef RLAMD_POOL_LREC
#define RLAMD_POOL_LREC 1
#endif
__host__ __device__ constexpr uint32_t pool_item_bytes() { return RLAMD_POOL_REC16 ? 16u : 10u; }
struct SmemLayout {
    uint32_t st, misc, q, sum, cnt, sfl, qf, n, nd, t, list, rcp, tr, cdf, lrec, trc, qd, rm, total;
    uint32_t trc_cap;   // pair traces: list slots per lane held in LDS (the rest in HBM)
    uint32_t nrcp;   // entries of the 1.0/n table (larger n: a division, same bits)
};
__host__ __device__ inline uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

// Blackjack's LDS rows (shared mode, eps-greedy): the learner group's Q copy holds
// only the states an update can write — non-terminal observations, p <= 21 and
// dealer card d <= 10 (blackjack.rs:121-162: every other observation ends the
// episode) — as (p*11 + d)*2 + ace, 484 of the 2048 dense rows.  Terminal rows
// are only read (TD target / selection at s'), never written, so they are read
// from Q_base in HBM (L2-resident).  UCB writes counters at terminal s' too, so
// UCB keeps the dense rows.
constexpr uint32_t BJ_LDS_STATES = 22u * 11u * 2u;
__host__ __device__ inline bool bj_compact(int env, int ucb) { return env == RL_ENV_BLACKJACK && !ucb; }
__host__ __device__ inline bool bj_nonterminal(uint32_t s) {
    const uint32_t p = s >> 6, d = (s >> 1) & 31u;
    return p <= 21u && d <= 10u;
}
__host__ __device__ inline uint32_t bj_row(uint32_t s) {          // dense obs -> LDS row
    const uint32_t p = s >> 6, r = s & 63u;
    return (p * 11u + (r >> 1)) * 2u + (r & 1u);
}
__host__ __device__ inline uint32_t bj_dense(uint32_t row) {      // LDS row -> dense obs
    const uint32_t pd = row >> 1, p = pd / 11u, d = pd - p * 11u;
    return ((p << 5) + d) * 2u + (row & 1u);
}
// Pair traces on small tables (FrozenLake, CliffWalking: S*A <= 256, so a pair id
// is 8 bits) keep every wave's visited pairs in one pool (pair_pool below)
__host__ __device__ constexpr bool pair_pool_env(int env) {
    return env == RL_ENV_CLIFF_WALKING || env == RL_ENV_FROZEN_LAKE || env == RL_ENV_FROZEN_LAKE_EDITED;
}
// Fixed-point single-table Q-learning (rl_device.h argmax_max, the fused argmax +
// max of the target row) keeps an f64 image of every entry beside its int64 word:
// the step reads values (selection, TD target, Q(s,a)) without converting, and
// the settle, the only writer, converts once per changed entry.
#ifndef RLAMD_NF_SKIP
#define RLAMD_NF_SKIP 1   // f64 one-step: no pass-2 count for entries with non-finite contributions
#endif
#ifndef RLAMD_LATE_B3
#define RLAMD_LATE_B3 1   // the step-separating barrier after the next step's env step
#endif
#ifndef RLAMD_TAXI_PF
#define RLAMD_TAXI_PF 1   // Taxi: the next step's transition word read from the HBM table after the selection
#endif
#ifndef RLAMD_TRPF
#define RLAMD_TRPF 0   // 1: FrozenLake reads the next step's transition word after the selection
                       // (cfg 2: 0.2122-0.2139 ms against 0.2116-0.2125 without, A/B on one box)
#endif
#ifndef RLAMD_EARLY_COUNT
#define RLAMD_EARLY_COUNT 0   // 1: count the step's train / episode-end lanes where their masks form (cfg 2: 147 static VALU against 144)
#endif
#ifndef RLAMD_TAIL
#define RLAMD_TAIL 0   // 1: the throughput kernels' end-of-step bookkeeping as one predicated
                       // block (cfg 2: 0.2149-0.2157 ms against 0.2139-0.2145, A/B on one box)
#endif
#ifndef RLAMD_QSH
#define RLAMD_QSH 2   // 0: off; 1: row reads as the compiler picks (ds_read2_b64: 0.2574 ms on cfg 2);
                      // 2: rows as 16-byte reads (0.2156 ms; no shadow 0.2206 ms)
#endif
__host__ __device__ constexpr bool qsh_layout(int fq, int ucb, int P, int algo) {
    return RLAMD_QSH != 0 && RLAMD_FUSE_MAX != 0 && !fq && !ucb && P == 1 && algo == RL_ALGO_QLEARNING;
}
// Row summaries (the QSH layout, rows of 4 actions): RM[s] = (max, argmax) of row
// s, written by the settle for every row each step, so a step reads its target
// row's argmax (the exploit action) and max (the Q-learning target) as one 16-byte
// LDS read instead of the 32-byte row and the 4-way compare chain.  The settle
// then runs on 2 of a group's 8 waves, each thread two entries of a row, with the
// row's halves combined across lane pairs (DPP).
#ifndef RLAMD_ROWMAX
#define RLAMD_ROWMAX 1
#endif
#ifndef RLAMD_RM_PIN
#define RLAMD_RM_PIN 0
#endif
#ifndef RLAMD_QA_EARLY
#define RLAMD_QA_EARLY 1   // rmx: Q(s, a) for the TD read right after the barrier, beside the row summary
#endif
#ifndef RLAMD_RSUM_REG
#define RLAMD_RSUM_REG 0   // 1: training-episode rewards summed per lane in registers, one LDS add per wave
                           // at launch end (cfg 2: 0.1929 against 0.1896 ms per launch, A/B on one box)
#endif
#ifndef RLAMD_RUN_TRAIN
#define RLAMD_RUN_TRAIN 0  // 1: throughput mode takes train == doS (a live lane is always in TRAIN mode);
                           // with RSUM_REG 0.1903 ms, no gain
#endif
#ifndef RLAMD_QA_EARLY2
#define RLAMD_QA_EARLY2 1   // traces (not UCB + expected SARSA): Q(s, a) read early (cfg 4: 0.5377 -> 0.5339 ms;
                            // on cfg 5's one-step double tables it measured 0.3528 -> 0.3549: not used there)
#endif
#ifndef RLAMD_SETTLE_RCPN
#define RLAMD_SETTLE_RCPN 0   // 1: the settle's 1/n by v_rcp_f64 + one Newton step, no table read
#endif
#ifndef RLAMD_SETTLE_QUAD
#define RLAMD_SETTLE_QUAD 1   // 1: one entry per thread (4 waves), the row summary by 2 DPP steps per quad
#endif
// LDS carve of one learner group (shared mode) or of the tables only (private).
//   misc u32[4]            f64 traces: the group step's max td code
//   q    int64 [P][S][A]   the group's Q copy (fixed point 2^-40, or f64 bits)
//   sum  int64 [P][S][A]   this step's summed contributions per entry (integers:
//                          the fixed point's units, or the f64 entry's grid)
//   cnt  fixed point: u16 [P][S][A] contributions per entry (u32-word atomics);
//        f64 one-step: u32 [P][S][A] = kinds of non-finite contributions << 28 |
//        (max code + 1) << 16 | count; traces: u32 per (table, row) counts
//   sfl  u8  [P][S][A]     f64 traces: kinds of this step's non-finite contributions
//                          (UCB + expected SARSA: bits 4-6 of qf instead)
//   qf   u8  [P][S][A]     UCB + expected SARSA: visible NaN/+-inf kinds of the entries
//   n/t  UCB counters (u64 [S][A], u64 t);  list u16 touched rows + count (traces)
//   rcp  f64 [nthr+1]   1.0/n for the combination rule (mean_delta)
//   tr   env transition table (FrozenLake / CliffWalking; Taxi computes its
//        transitions and reads its start cdf from HBM, Blackjack has none)
//   trc  pair traces (traces == 2): the first trc_cap slots of every lane's pair
//        list, ids u16 [cap][nthr] then E f64 [cap][nthr] (column = thread);
//        small tables: the first trc_cap items of every wave's pair pool
// nthr = the shared kernel's block size; 0 for the private kernel (tables only).
// traces: 0 none, 1 whole-row visited-state sets, 2 visited-pair sets
// ucb: 0 none, 1 UCB, 2 UCB + expected SARSA (launch counts u32 [S][A] + step
// counts u16 [S][A], or both in one u32 when ucb_pack)
__host__ __device__ inline SmemLayout smem_layout(int env, int P, int ucb, int traces, uint32_t S,
                                                  uint32_t A, uint32_t n_start, uint32_t nthr,
                                                  uint32_t trc_kb = 40u, int fq = 0, int ucb_pack = 0,
                                                  int qsh = 0) {
    const int shared_q = nthr != 0;
    SmemLayout l;
    const uint32_t SL = (shared_q && bj_compact(env, ucb)) ? BJ_LDS_STATES : S;   // LDS rows
    const uint32_t SA = S * A, PSA = (uint32_t)P * SL * A;
    // full 1.0/n table when every entry is settled each step (sweep form: n can
    // reach the group size); 64 entries for the owner form (few contributions)
    l.nrcp = !shared_q ? 0u : (PSA <= nthr ? nthr + 1u : (nthr + 1u < 65u ? nthr + 1u : 65u));
    uint32_t off = 0;
    l.st = off; off += STATS_W * 8u;              // per-block stats accumulators (u64[STATS_W])
    l.misc = off; off += shared_q ? 16u : 0u;
    l.q = off; off += shared_q ? align16(PSA * 8u) : 0u;
    l.sum = off; off += shared_q ? align16(PSA * 8u) : 0u;
    l.cnt = off; off += shared_q ? align16((fq && !traces) ? PSA * 4u : ((PSA + 1u) / 2u) * 4u) : 0u;
    l.sfl = off; off += (shared_q && fq && traces && ucb != 2) ? align16(((PSA + 3u) / 4u) * 4u) : 0u;
    l.qf = off; off += (shared_q && ucb == 2) ? align16(((PSA + 3u) / 4u) * 4u) : 0u;
    l.n = off;
    l.nd = off + align16(SA * 4u);
    off += (shared_q && ucb)
               ? (ucb == 2 ? (ucb_pack ? align16(SA * 4u) : align16(SA * 4u) + align16(((SA + 1u) / 2u) * 4u))
                           : align16(SA * 8u))
               : 0u;
    l.t = off; off += (shared_q && ucb) ? (ucb == 2 ? 32u : 16u) : 0u;   // T[0], T[1] (+ ARR: UCB + ES)
    l.list = off; off += (shared_q && traces) ? align16(PSA * 2u) + 16u : 0u;
    l.rcp = off; off += align16(l.nrcp * 8u);
    l.tr = off; off += (env == RL_ENV_TAXI || env == RL_ENV_BLACKJACK) ? 0u : align16(SA * 4u);
    // start distributions: FrozenLake's maps start at 0 (fixed_start), Taxi probes
    // the HBM cdf (taxi_start), CliffWalking / Blackjack have none
    (void)n_start;
    l.cdf = off;
    // trc_kb KiB per group (KParams::trc_kb), at most S*A slots per lane
    // row strides padded by 2 / 1 entries (PairCache): one lane's consecutive
    // slots then sit in different LDS banks
    // pool form (small tables, pair_pool): trc_cap = items per wave, tags u16
    // [waves][cap] then E f64 [waves][cap]
    const bool pool = shared_q && traces == 2 && pair_pool_env(env);
    // RLAMD_POOL_LREC: the pool sweep's per-lane record {td, pk} (16 B per lane of
    // every wave), read by the items instead of three shuffles
    l.lrec = off;
    if (pool && RLAMD_POOL_LREC) off += (nthr >> 6) * 64u * 16u;
    if (pool) {
        const uint32_t nw = nthr >> 6, c = trc_kb * 1024u / (nw * pool_item_bytes());
        l.trc_cap = c < 64u * S * A ? c : 64u * S * A;
    } else if (shared_q && traces == 2) {
        const uint32_t c = trc_kb * 1024u / ((nthr + 2u) * 2u + (nthr + 1u) * 8u);
        l.trc_cap = c < S * A ? c : S * A;
    } else {
        l.trc_cap = 0u;
    }
    l.trc = off;
    if (pool && RLAMD_POOL_REC16) off += l.trc_cap * (nthr >> 6) * 16u;
    else if (pool) off += l.trc_cap ? align16(l.trc_cap * (nthr >> 6) * 2u) + l.trc_cap * (nthr >> 6) * 8u : 0u;
    else off += l.trc_cap ? align16(l.trc_cap * (nthr + 2u) * 2u) + l.trc_cap * (nthr + 1u) * 8u : 0u;
    // qd  f64 [P][S][A]  fixed-point single-table Q-learning: the f64 image of every
    //                    entry beside its int64 word (qsh_layout), read by the step
    if (shared_q && qsh) off = align16(off);
    l.qd = off; off += (shared_q && qsh) ? PSA * 8u : 0u;
    off = align16(off);
    l.rm = off; off += (shared_q && qsh && RLAMD_ROWMAX && A == 4u && P == 1) ? SL * 16u : 0u;
    l.total = off;
    return l;
}

// The shared-mode combination rule (oracle: rlref.c mean_delta): an entry moves
// by the MEAN of the n contributions it received, trunc((double)sum * (1.0/n))
// with 1.0/n correctly rounded (rcp[0] = 0, rcp[1] = 1: n <= 1 is exact).
// The device form reads 1.0/n from the LDS table and converts with the
// 1.5*2^52 magic add (|mean| <= 2^51 for step contributions).
__host__ __device__ inline int64_t mean_delta(int64_t sum, int64_t n) {
    if (n <= 0) return 0;
    return (int64_t)__builtin_trunc((double)sum * (1.0 / (double)n));
}
__device__ __forceinline__ int64_t mean_delta_rcp(int64_t sum, double rcp) {
    const double y = __builtin_trunc((double)sum * rcp) + 0x1.8p52;
    return (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull);
}

// ---------------------------------------------------------------- lane state
struct LaneRegs {
    Rng rng;
    uint32_t s, a, z, train_ep, eval_left, epi_len;
    uint32_t mode;
    bool need_reset, ready, dflag;
    double eps, epi_reward;
};
// per-launch counters (rl_stats slots 0-4); the shared kernel keeps them per
// wave in scalar registers (ballot counts), the private kernel per lane
struct Counters {
    uint32_t n_train = 0, n_eval = 0, n_tep = 0, n_eep = 0;
    int64_t rsum = 0;      // sum over finished training episodes of rint(reward * 2^16)
    uint32_t trace_states = 0;   // visited-set entries swept by the eligibility update
};


__device__ __forceinline__ void lane_load(const KParams &p, uint64_t lane, bool active, LaneRegs &L) {
    uint4 c = make_uint4(0, 0, 0, 0), r = make_uint4(1, 0, 0, 0), x = make_uint4(0, 0, 0, 0);
    double er = 0.0;
    if (active) { c = p.core[lane]; r = p.rng[lane]; x = p.aux[lane]; er = p.epi_reward[lane]; }
    L.rng.s0 = r.x; L.rng.s1 = r.y; L.rng.s2 = r.z; L.rng.s3 = r.w;
    L.s = c.x;
    L.a = c.y & LF_ACT_MASK;
    L.need_reset = (c.y & LF_NEED_RESET) != 0;
    L.ready = (c.y & LF_READY) != 0;
    L.dflag = (c.y & LF_DFLAG) != 0;
    L.mode = active ? (c.y >> LF_MODE_SHIFT) & 3u : (uint32_t)RL_MODE_DONE;
    L.z = c.z;
    L.train_ep = c.w;
    L.eps = __longlong_as_double((long long)(((uint64_t)x.y << 32) | x.x));
    L.eval_left = x.z;
    L.epi_len = x.w;
    L.epi_reward = er;
}
__device__ __forceinline__ void lane_store(const KParams &p, uint64_t lane, const LaneRegs &L) {
    const uint32_t y = (L.a & LF_ACT_MASK) | (L.need_reset ? LF_NEED_RESET : 0u) |
                       (L.ready ? LF_READY : 0u) | (L.dflag ? LF_DFLAG : 0u) |
                       (L.mode << LF_MODE_SHIFT);
    p.core[lane] = make_uint4(L.s, y, L.z, L.train_ep);
    p.rng[lane] = make_uint4(L.rng.s0, L.rng.s1, L.rng.s2, L.rng.s3);
    const uint64_t e = (uint64_t)__double_as_longlong(L.eps);
    p.aux[lane] = make_uint4((uint32_t)e, (uint32_t)(e >> 32), L.eval_left, L.epi_len);
    p.epi_reward[lane] = L.epi_reward;
}

// per-launch counters -> rl_stats: wave sums -> block sums in LDS (acc) -> one
// atomic per block and counter into stats replica blockIdx % STATS_REP.
// Every thread of the block must call these (they contain a barrier).
__device__ __forceinline__ void flush_block(const KParams &p, unsigned long long *acc) {
    __syncthreads();
    if (threadIdx.x < STATS_W && threadIdx.x != 6 && acc[threadIdx.x])
        atomicAdd(&p.stats[(blockIdx.x % STATS_REP) * STATS_W + threadIdx.x], acc[threadIdx.x]);
}
__device__ __forceinline__ void flush_stats(const KParams &p, const LaneRegs &L, const Counters &C,
                                            bool active, unsigned long long *acc) {
    const uint64_t v[8] = {C.n_train, C.n_eval, C.n_tep, C.n_eep, (uint64_t)C.rsum,
                           (uint64_t)(active && L.mode == RL_MODE_DONE), 0, C.trace_states};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (i == 6) continue;
        const int64_t s = wave_sum_i64((int64_t)v[i]);
        if ((threadIdx.x & 63u) == 0 && s != 0) atomicAdd(&acc[i], (unsigned long long)s);
    }
    flush_block(p, acc);
}
// 1 when the episode index is a multiple of eval_at (src/agent.rs:107):
// Lemire's divisibility test, ep * c <= c - 1 (mod 2^64) with c = ceil(2^64 / eval_at)
// precomputed on the host (eval_div; 0 for eval_at == 1, every episode).
__device__ __forceinline__ bool eval_hit(const KParams &p, uint32_t ep) {
    return p.eval_at != 0 && (uint64_t)ep * p.eval_div <= p.eval_div - 1ull;
}

// bookkeeping after the update: src/agent.rs:98-116 + the eval interleave.
// Written as predicated selects (no divergent branches): lanes end episodes at
// different steps, and the branchy form was mis-scheduled at -O3 (a lost
// train_ep increment, caught by the parity tests).
// Sets tr / ev when a training / evaluation episode ended (the caller counts them).
// EPI: 0 = throughput mode compiled in (no target, no eval interleave: rl_agent_run),
// 1 = episodic, -1 = KParams::episodic at run time
template <int EPI = -1>
__device__ __forceinline__ void after_step(const KParams &p, LaneRegs &L, uint32_t s2, uint32_t a2,
                                           double r, bool term, bool &tr_out, bool &ev_out) {
    L.epi_reward += r;
    L.epi_len += 1;
    L.s = s2;
    L.a = a2;
    const bool tr = term && L.mode == RL_MODE_TRAIN;
    const bool ev = term && L.mode == RL_MODE_EVAL;
    tr_out = tr;
    ev_out = ev;
    if (EPI == 0 || (EPI < 0 && !p.episodic)) {   // throughput mode (rl_agent_run): no target, no eval interleave;
        // the general logic below reduces to exactly this
        L.train_ep += tr ? 1u : 0u;
        const uint32_t el = L.eval_left - (ev ? 1u : 0u);
        L.mode = (ev && el == 0u) ? (uint32_t)RL_MODE_TRAIN : L.mode;
        L.eval_left = el;
        L.need_reset = L.need_reset || term;
        return;
    }
    const uint32_t ep = L.train_ep;                      // index of the episode that just ended
    const uint32_t new_ep = ep + (tr ? 1u : 0u);
    const bool go_eval = tr && p.eval_episodes != 0 && eval_hit(p, ep);   // episode % eval_at == 0
    const bool reached = p.target_episodes != 0 && (uint64_t)new_ep >= p.target_episodes;
    const bool tr_done = tr && !go_eval && reached;
    const uint32_t el = L.eval_left - (ev ? 1u : 0u);
    const bool ev_end = ev && el == 0u;
    const bool ev_fin = p.eval_only != 0 || reached;
    uint32_t mode = L.mode;
    mode = go_eval ? (uint32_t)RL_MODE_EVAL : mode;
    mode = tr_done ? (uint32_t)RL_MODE_DONE : mode;
    mode = ev_end ? (ev_fin ? (uint32_t)RL_MODE_DONE : (uint32_t)RL_MODE_TRAIN) : mode;
    L.mode = mode;
    L.train_ep = new_ep;
    L.eval_left = go_eval ? p.eval_episodes : el;
    L.need_reset = L.need_reset || term;
}

// episode log: reward_history / episode_length entries (src/agent.rs:96-100,
// :131-138).  The per-lane count lives in HBM and is touched only at episode
// end, so the step loop carries no extra register.
__device__ __forceinline__ void log_episode(const KParams &p, uint64_t lane, const LaneRegs &L, bool train_ep) {
    const uint32_t c = p.elog_cnt[lane];
    rl_episode_record e;
    e.lane = (uint32_t)lane;
    e.length = L.epi_len;
    e.seq = c;
    e.mode = train_ep ? (uint8_t)RL_MODE_TRAIN : (uint8_t)RL_MODE_EVAL;
    e.pad[0] = e.pad[1] = e.pad[2] = 0;
    e.reward = L.epi_reward;
    p.elog[(uint64_t)(c % p.elog_cap) * p.L + lane] = e;
    p.elog_cnt[lane] = c + 1u;
}

__device__ __forceinline__ void write_record(const KParams &p, uint32_t k, uint64_t lane, uint32_t kind,
                                             uint32_t s, uint32_t a, uint32_t s2, uint32_t a2, double r,
                                             bool term, double td, uint32_t mode) {
    rl_step_record rec;
    rec.s = s;
    rec.s2 = s2;
    rec.a = (uint8_t)a;
    rec.a2 = (uint8_t)a2;
    rec.term = (uint8_t)term;
    rec.mode = (uint8_t)mode;
    rec.kind = (uint8_t)kind;
    rec.pad[0] = rec.pad[1] = rec.pad[2] = 0;
    rec.r = r;
    rec.td = td;
    p.rec[(uint64_t)k * p.L + lane] = rec;
}

// E[s][a] += 1 (elegibility_traces_agent.rs:75-80): find s in the lane's sparse
// set or append it with a fresh zero row (slot-major SoA, coalesced per slot)
template <int A>
__device__ __forceinline__ void trace_visit(const KParams &p, uint64_t lane, uint32_t s, uint32_t a,
                                            uint32_t &cnt) {
    const uint64_t Ls = p.L;
    uint32_t j = p.slot_of[(uint64_t)s * Ls + lane];
    if (j < cnt && p.tlist[(uint64_t)j * Ls + lane] == s) {
        double *e = &p.trace[((uint64_t)j * A + a) * Ls + lane];
        *e = *e + 1.0;
    } else {
        j = cnt++;
        p.tlist[(uint64_t)j * Ls + lane] = (uint16_t)s;
        p.slot_of[(uint64_t)s * Ls + lane] = (uint16_t)j;
#pragma unroll
        for (int b = 0; b < A; ++b) p.trace[((uint64_t)j * A + b) * Ls + lane] = (uint32_t)b == a ? 1.0 : 0.0;
    }
}

// The eligibility sweep over slots [0, nv): E[o][b] is read, fn(o, b, E) applied,
// E *= gamma*lambda written back.  TC slots at a time with every load issued
// before any use (memory-level parallelism; slot j of all lanes is one row).
template <int A, class RowFn, class Fn>
__device__ __forceinline__ void trace_sweep(const KParams &p, uint64_t lane, uint32_t nv, RowFn &&row_fn, Fn &&fn) {
    constexpr uint32_t TC = 4;
    const uint64_t Ls = p.L;
    for (uint32_t j0 = 0; j0 < nv; j0 += TC) {
        uint32_t o[TC];
        double ev[TC][A];
#pragma unroll
        for (uint32_t c = 0; c < TC; ++c) {
            const bool in = j0 + c < nv;
            const uint32_t j = in ? j0 + c : j0;
            o[c] = p.tlist[(uint64_t)j * Ls + lane];
#pragma unroll
            for (int b = 0; b < A; ++b) ev[c][b] = p.trace[((uint64_t)j * A + b) * Ls + lane];
        }
#pragma unroll
        for (uint32_t c = 0; c < TC; ++c) {
            if (j0 + c < nv) {
                const uint32_t j = j0 + c;
                row_fn(o[c]);
#pragma unroll
                for (int b = 0; b < A; ++b) {
                    fn(o[c], (uint32_t)b, ev[c][b]);
                    p.trace[((uint64_t)j * A + b) * Ls + lane] = ev[c][b] * p.gl;
                }
            }
        }
    }
}

// Shared-mode traces over visited (state, action) PAIRS (layout_sparse_traces).
// Slot j of a lane's list holds pair id s*A+a (| 0x8000 on the first pair of its
// state this episode: the state joins the visited set, its row is counted once
// per step, as the reference updates every action of it) and E of the pair.
// Slots j < cap live in LDS (TRI ids / TRE values, column = thread) for the
// launch and are found by a scan; slots j >= cap live in HBM (tlist / trace
// [j][L]) with slot_of [id][L] and the visited-state bitmap vbits for them.
#ifndef RLAMD_PLAN_PB
#define RLAMD_PLAN_PB 16   // Dyna planning steps whose draws and model reads go out together
#endif
#ifndef RLAMD_PLAN_PF
#define RLAMD_PLAN_PF 1   // Dyna planning (eps-greedy): a batch's draws first, its model reads together
#endif
#ifndef RLAMD_LAZY_ROWS
#define RLAMD_LAZY_ROWS 1   // reset-and-step: the reset's selection reads its row only for exploiting lanes
#endif
#ifndef RLAMD_BJ_ONE_LOOP
// Blackjack learner groups: reset and step draws in one loop (EnvDev::advance).
// Parity-green but measured slower on cfg 5 (4.98e10 vs 5.83e10 env-steps/s on
// the 8-wave kernel), so off
#define RLAMD_BJ_ONE_LOOP 0
#endif

#ifndef RLAMD_SWEEP_U
#define RLAMD_SWEEP_U 4   // pair-trace sweep: rounds of 64 items interleaved per iteration
                          // (cfg 4: 1 / 2 / 4 -> 1.163 / 1.089 / 1.058 ms per launch)
#endif
#ifndef RLAMD_COOP_SWEEP
#define RLAMD_COOP_SWEEP 1   // shared pair traces: wave-cooperative sweep (0: each lane its own list)
#endif
#ifndef RLAMD_PAIR_BITS
#define RLAMD_PAIR_BITS 1   // small tables: visited-pair bitmap in registers (0: scan the list)
#endif
#ifndef RLAMD_TRACES_W
#define RLAMD_TRACES_W 0   // small-table traces at <= 2 groups per CU: a 256-VGPR kernel
                           // (measured equal on cfg 4 once the bitmap and opq() removed the
                           // scratch arrays: 0.8875 vs 0.8869 ms, so off)
#endif
#ifndef RLAMD_OWNER_SCAN
#define RLAMD_OWNER_SCAN 1   // pair-trace sweep: item owners by ballot + readlane scan (0: shuffle binary search)
#endif
#ifndef RLAMD_PAIR_TC
#define RLAMD_PAIR_TC 8   // HBM pair slots per batch of the sweep (loads issued together)
#endif
// HBM pair slots (those past the LDS cache): lane-major, [lane][j] with stride S*A
// (the longest list), so the consecutive items of one lane a sweep round takes
// are contiguous — one or two cache lines instead of one line per item
#ifndef RLAMD_PAIR_LANE_MAJOR
#define RLAMD_PAIR_LANE_MAJOR 1   // 0: slot-major [j][lane]
#endif
__device__ __forceinline__ uint64_t pslot(const KParams &p, uint32_t j, uint64_t lane) {
    if constexpr (RLAMD_PAIR_LANE_MAJOR) return lane * (uint64_t)(p.S * p.A) + j;
    else return (uint64_t)j * p.L + lane;
}
struct PairCache {
    uint16_t *TRI;
    double *TRE;
    uint32_t cap, nthr, tid;
    // slot j of thread t: ids in rows of nthr + 2 u16, E in rows of nthr + 1 f64 —
    // unpadded, a lane's slots j, j+1, ... (what one sweep round reads) were
    // 2 KiB apart for 256 threads, i.e. all in one LDS bank
    __device__ __forceinline__ uint32_t ixi_t(uint32_t j, uint32_t t) const { return j * (nthr + 2u) + t; }
    __device__ __forceinline__ uint32_t ixe_t(uint32_t j, uint32_t t) const { return j * (nthr + 1u) + t; }
    __device__ __forceinline__ uint32_t ixi(uint32_t j) const { return ixi_t(j, tid); }
    __device__ __forceinline__ uint32_t ixe(uint32_t j) const { return ixe_t(j, tid); }
};
// E[s][a] += 1: find the pair or append it
template <int A>
__device__ __forceinline__ void pair_visit(const KParams &p, const PairCache &c, uint64_t lane, uint32_t s,
                                           uint32_t a, uint32_t &np) {
    const uint64_t Ls = p.L;
    const uint32_t id = s * (uint32_t)A + a, id0 = s * (uint32_t)A;
    const uint32_t nl = np < c.cap ? np : c.cap;
    uint32_t hit = 0xffffffffu;
    bool same_state = false;
    constexpr uint32_t TB = 8;                      // ids read TB at a time (latency)
    for (uint32_t j0 = 0; j0 < nl; j0 += TB) {
        uint32_t w[TB];
#pragma unroll
        for (uint32_t k = 0; k < TB; ++k) w[k] = c.TRI[c.ixi(j0 + k < nl ? j0 + k : j0)] & 0x7fffu;
#pragma unroll
        for (uint32_t k = 0; k < TB; ++k) {
            if (j0 + k < nl) {
                if (w[k] == id) hit = j0 + k;
                if (w[k] - id0 < (uint32_t)A) same_state = true;
            }
        }
    }
    if (hit != 0xffffffffu) {
        c.TRE[c.ixe(hit)] += 1.0;
        return;
    }
    if (np > c.cap) {                               // overflow part: slot_of lookup
        const uint32_t j = p.slot_of[(uint64_t)id * Ls + lane];
        if (j >= c.cap && j < np && (p.tlist[pslot(p, j, lane)] & 0x7fffu) == id) {
            double *e = &p.trace[pslot(p, j, lane)];
            *e = *e + 1.0;
            return;
        }
    }
    const uint32_t j = np++;
    if (j < c.cap) {
        c.TRI[c.ixi(j)] = (uint16_t)(id | (same_state ? 0u : 0x8000u));
        c.TRE[c.ixe(j)] = 1.0;
    } else {
        uint32_t *vw = &p.vbits[(uint64_t)(s >> 5) * Ls + lane];
        const uint32_t vb = *vw, bit = 1u << (s & 31u);
        const bool first = !same_state && (vb & bit) == 0u;
        if ((vb & bit) == 0u) *vw = vb | bit;
        p.tlist[pslot(p, j, lane)] = (uint16_t)(id | (first ? 0x8000u : 0u));
        p.slot_of[(uint64_t)id * Ls + lane] = (uint16_t)j;
        p.trace[pslot(p, j, lane)] = 1.0;
    }
}
// the sweep over pairs [0, np): fn(pair id, first-of-state, E); E *= gamma*lambda.
// LDS slots first, then the HBM slots TC at a time with every load issued first.
template <class Fn>
__device__ __forceinline__ void pair_sweep(const KParams &p, const PairCache &c, uint64_t lane, uint32_t np,
                                           Fn &&fn) {
    const uint32_t nl = np < c.cap ? np : c.cap;
    constexpr uint32_t TL = 4;                      // LDS slots read TL at a time (latency)
    for (uint32_t j0 = 0; j0 < nl; j0 += TL) {
        uint32_t w[TL];
        double ev[TL];
#pragma unroll
        for (uint32_t k = 0; k < TL; ++k) {
            const uint32_t j = j0 + k < nl ? j0 + k : j0;
            w[k] = c.TRI[c.ixi(j)];
            ev[k] = c.TRE[c.ixe(j)];
        }
#pragma unroll
        for (uint32_t k = 0; k < TL; ++k) {
            if (j0 + k < nl) {
                fn(w[k] & 0x7fffu, (w[k] & 0x8000u) != 0u, ev[k]);
                c.TRE[c.ixe(j0 + k)] = ev[k] * p.gl;
            }
        }
    }
    constexpr uint32_t TC = RLAMD_PAIR_TC;
    for (uint32_t j0 = c.cap; j0 < np; j0 += TC) {
        uint32_t w[TC];
        double ev[TC];
#pragma unroll
        for (uint32_t k = 0; k < TC; ++k) {
            const uint32_t j = j0 + k < np ? j0 + k : j0;
            w[k] = p.tlist[pslot(p, j, lane)];
            ev[k] = p.trace[pslot(p, j, lane)];
        }
#pragma unroll
        for (uint32_t k = 0; k < TC; ++k) {
            if (j0 + k < np) {
                fn(w[k] & 0x7fffu, (w[k] & 0x8000u) != 0u, ev[k]);
                p.trace[pslot(p, j0 + k, lane)] = ev[k] * p.gl;
            }
        }
    }
}
// the episode ended: the list is emptied by np = 0; the bitmap (set only by
// HBM-slot appends) is cleared when the list had reached them
__device__ __forceinline__ void pair_clear(const KParams &p, const PairCache &c, uint64_t lane, uint32_t np) {
    if (np <= c.cap) return;
    const uint32_t nw = (p.S + 31u) >> 5;
    for (uint32_t w = 0; w < nw; ++w) p.vbits[(uint64_t)w * p.L + lane] = 0u;
}
// launch boundaries: LDS slots <-> tlist / trace rows (np persists in p.tcnt)
__device__ __forceinline__ void pair_cache_load(const KParams &p, const PairCache &c, uint64_t lane, uint32_t np) {
    const uint32_t nl = np < c.cap ? np : c.cap;
    for (uint32_t j = 0; j < nl; ++j) {
        c.TRI[c.ixi(j)] = p.tlist[pslot(p, j, lane)];
        c.TRE[c.ixe(j)] = p.trace[pslot(p, j, lane)];
    }
}
__device__ __forceinline__ void pair_cache_store(const KParams &p, const PairCache &c, uint64_t lane, uint32_t np) {
    const uint32_t nl = np < c.cap ? np : c.cap;
    for (uint32_t j = 0; j < nl; ++j) {
        p.tlist[pslot(p, j, lane)] = c.TRI[c.ixi(j)];
        p.trace[pslot(p, j, lane)] = c.TRE[c.ixe(j)];
    }
}

// UCB + expected SARSA: the visible NaN/+-inf kinds of every entry (bits 0-2 of
// QF8, the kinds of the entry's f64 value) let a lane decide the F7 regime from
// one two-word row read.  A step's non-finite contributions are ORed into bits
// 4-6 (the f64 step kinds, SFL below) while other waves may still read the row;
// the entry's settle, after every reader of the step, writes the new value and
// its visible kinds.
constexpr uint32_t QF_MASK = QF_NAN | QF_PINF | QF_NINF, QF_PENDING = 4u;
__device__ __forceinline__ uint32_t value_flags(double q) { return __builtin_isfinite(q) ? 0u : nf_flag(q); }

// the fixed point is only ever run where the host's range proof can hold
// (rl_host.cpp delta_bound): one-step agent, single table, contracting bootstrap
template <int AGENT, int POLICY, int SEL, int ALGO>
constexpr bool fix_possible() {
    return AGENT == RL_AGENT_ONE_STEP && POLICY == RL_POLICY_TABULAR &&
           !(SEL == RL_SEL_UCB && ALGO == RL_ALGO_EXPECTED_SARSA);
}

// ======================================================================== shared
// INSTR: step records / episode log compiled in (chosen at launch when either is
// enabled); the throughput variant carries neither.
// FQ: the group's Q is f64 (rl_device.h "f64 shared Q"); else the fixed point,
// which the host runs only where it proved the range (no clamp can engage).
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, bool INSTR, bool FQ, int SLIP = -1, int SWEEP = -1,
          bool PACK = false, int RS = -1, int EPI = -1>
__device__ __forceinline__ void train_shared_body(const KParams &p) {
    using E = EnvDev<ENV>;
    constexpr int A = E::A;
    constexpr int P = POLICY == RL_POLICY_DOUBLE ? 2 : 1;
    constexpr bool UCB = SEL == RL_SEL_UCB;
    constexpr bool TRACES = AGENT == RL_AGENT_TRACES;
    constexpr bool SPEC = UCB && ALGO == RL_ALGO_EXPECTED_SARSA;  // inf/NaN possible
    static_assert(FQ || fix_possible<AGENT, POLICY, SEL, ALGO>(), "no range proof: f64 only");
    constexpr bool BJC = ENV == RL_ENV_BLACKJACK && !UCB;   // compact LDS rows (bj_row)
    const uint32_t S = p.S, SA = S * (uint32_t)A, PSA = (uint32_t)P * SA;
    const uint32_t SL = BJC ? BJ_LDS_STATES : S, SAL = SL * (uint32_t)A, PSAL = (uint32_t)P * SAL;

    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    constexpr bool PAIRS = TRACES && !SPEC;            // layout_sparse_traces (rl_kparams.h)
    constexpr bool QSH = qsh_layout(FQ ? 1 : 0, UCB ? 1 : 0, P, ALGO);
    const SmemLayout lay = smem_layout(ENV, P, UCB ? (SPEC ? 2 : 1) : 0, TRACES ? (PAIRS ? 2 : 1) : 0, S, A, p.n_start,
                                       nthr, p.trc_kb, FQ ? 1 : 0, p.ucb_pack, QSH ? 1 : 0);
    unsigned long long *Q = (unsigned long long *)(smem + lay.q);
    double *QD = (double *)(smem + lay.qd);              // QSH: f64 images of Q's words
    double2 *RM = (double2 *)(smem + lay.rm);            // QSH rows of 4: (max, argmax bits) per row
    unsigned long long *SUM = (unsigned long long *)(smem + lay.sum);
    uint32_t *CNT = (uint32_t *)(smem + lay.cnt);        // fixed point: two u16 counters per word
    uint16_t *CNT16 = (uint16_t *)(smem + lay.cnt);
    uint32_t *W = (uint32_t *)(smem + lay.cnt);          // f64 one-step: kinds << 28 | max code + 1 << 16 | count
    // f64 traces: kinds of the step's non-finite contributions (own bytes; QF's bits 4-6 for SPEC)
    uint32_t *SFLW = (uint32_t *)(smem + (SPEC ? lay.qf : lay.sfl));
    uint8_t *SFL8 = (uint8_t *)(smem + (SPEC ? lay.qf : lay.sfl));
    constexpr uint32_t SFL_SH = SPEC ? QF_PENDING : 0u;
    uint32_t *QF = (uint32_t *)(smem + lay.qf);          // four u8 flag sets per word
    uint8_t *QF8 = (uint8_t *)(smem + lay.qf);
    unsigned long long *N = (unsigned long long *)(smem + lay.n);
    unsigned long long *T = (unsigned long long *)(smem + lay.t);
    // SPEC counters: n = n_base (HBM, u64) + NL (this launch) [+ D (this step)];
    // ucb_pack: NL = launch << 16 | step in one u32
    uint32_t *NL = (uint32_t *)(smem + lay.n);
    uint32_t *D32 = (uint32_t *)(smem + lay.nd);
    uint16_t *D16 = (uint16_t *)(smem + lay.nd);
    uint16_t *LIST = (uint16_t *)(smem + lay.list);
    uint32_t *LISTN = (uint32_t *)(smem + lay.list + align16(PSAL * 2u));
    uint32_t *TR = (uint32_t *)(smem + lay.tr);
    double *RCP = (double *)(smem + lay.rcp);
    uint32_t *GCODE = (uint32_t *)(smem + lay.misc);

    unsigned long long *ACC = (unsigned long long *)(smem + lay.st);
    // LDS table layout: state-major [tbl][s][a] like HBM (LDS_AM = false), or
    // action-major [tbl][a][s] (LDS_AM = true: measured 6 % slower on cfg 2 —
    // 4 ds_read_b64 per row instead of 2 ds_read_b128 cost more than the bank
    // conflicts they avoid).
    constexpr bool LDS_AM = false;
    auto lrow = [&](uint32_t s) -> uint32_t {
        if constexpr (BJC) return bj_row(s);
        else return s;
    };
    auto qi = [&](uint32_t tbl, uint32_t s, uint32_t a) -> uint32_t {
        return LDS_AM ? tbl * SAL + a * SL + lrow(s) : tbl * SAL + lrow(s) * (uint32_t)A + a;
    };
    auto dense_of = [&](uint32_t j) -> uint32_t {       // LDS Q index -> HBM [P][S][A] index
        if constexpr (!LDS_AM && !BJC) return j;
        const uint32_t tbl = j / SAL, r = j - tbl * SAL;
        const uint32_t row = LDS_AM ? r % SL : r / (uint32_t)A, a = LDS_AM ? r / SL : r % (uint32_t)A;
        const uint32_t s = BJC ? bj_dense(row) : row;
        return tbl * SA + s * (uint32_t)A + a;
    };
    auto lds_of = [&](uint32_t i) -> uint32_t {        // HBM index -> LDS index
        if constexpr (!LDS_AM) return i;
        const uint32_t tbl = i / SA, r = i - tbl * SA;
        return qi(tbl, r / (uint32_t)A, r % (uint32_t)A);
    };
    if (tid < STATS_W) ACC[tid] = 0ull;
    if (tid == 0) GCODE[0] = 0u;
    for (uint32_t i = tid; i < lay.nrcp; i += nthr) RCP[i] = i == 0 ? 0.0 : 1.0 / (double)i;
    for (uint32_t j = tid; j < PSAL; j += nthr) {
        Q[j] = (unsigned long long)p.q_base[dense_of(j)];
        SUM[j] = 0ull;
        if constexpr (QSH) QD[j] = q_val((int64_t)Q[j]);
    }
    if constexpr (FQ && !TRACES) {
        for (uint32_t j = tid; j < PSAL; j += nthr) W[j] = 0u;
    } else {
        for (uint32_t i = tid; i < (PSAL + 1u) / 2u; i += nthr) CNT[i] = 0u;
    }
    if constexpr (FQ && TRACES && !SPEC)
        for (uint32_t i = tid; i < (PSAL + 3u) / 4u; i += nthr) SFLW[i] = 0u;
    if constexpr (TRACES) { if (tid == 0) LISTN[0] = 0u; }
    if constexpr (UCB) {
        if constexpr (SPEC) {
            for (uint32_t j = tid; j < PSAL; j += nthr) QF8[j] = (uint8_t)value_flags(as_f64(Q[j]));
            for (uint32_t i = tid; i < SA; i += nthr) NL[i] = 0u;
            if (!p.ucb_pack)
                for (uint32_t i = tid; i < (SA + 1u) / 2u; i += nthr) D32[i] = 0u;
        } else {
            for (uint32_t i = tid; i < SA; i += nthr) N[lds_of(i)] = (unsigned long long)p.n_base[i];
        }
        if (tid == 0) {
            T[0] = p.t_base[0]; T[1] = 0ull;
            if constexpr (SPEC) *(uint32_t *)(T + 2) = 0u;
        }
    }
    if constexpr (ENV != RL_ENV_TAXI && ENV != RL_ENV_BLACKJACK)
        for (uint32_t i = tid; i < SA; i += nthr) TR[lds_of(i)] = p.trans[i];
    // row summaries (RLAMD_ROWMAX): in the sweep form only (the settle rewrites them)
    const bool sweep = SWEEP == 1 || PSAL <= nthr;   // SWEEP == 1: the host checked PSA <= block
    const bool rmx = QSH && RLAMD_ROWMAX && A == 4 && sweep;
    if (rmx) {
        for (uint32_t r = tid; r < SL; r += nthr) {
            double v[A], m;
#pragma unroll
            for (int i = 0; i < A; ++i) v[i] = q_val(p.q_base[r * (uint32_t)A + i]);
            const uint32_t a = argmax_max_f64<A>(v, m);
            RM[r] = make_double2(m, as_f64((uint64_t)a));
        }
    }
    __syncthreads();

    EnvTables tabs;
    tabs.trans = TR; tabs.cdf = p.start_cdf; tabs.n_start = p.n_start; tabs.max_steps = p.max_steps;
    tabs.th1 = p.th1; tabs.th2 = p.th2; tabs.th3 = p.th3; tabs.trunc_reward = p.trunc_reward;
    tabs.fixed_start = p.fixed_start;
    tabs.slippery = p.slippery;
    tabs.S = S;

    const uint32_t gl = (tid >> 6) * p.lpw + (tid & 63u);      // lane within the group (KParams::lpw)
    const uint64_t lane = (uint64_t)blockIdx.x * p.G + gl;
    const bool active = (tid & 63u) < p.lpw && gl < p.G && lane < p.L;
    LaneRegs L;
    lane_load(p, lane, active, L);
    uint32_t tcnt = 0, trace_states = 0;           // traces: size of the lane's visited set
    // UCB + expected SARSA: ln(t) once per step.  t changes only by the counter
    // increments between a step's selection and its probabilities, so the
    // probabilities' ln(t_{k+1}) is also step k+1's selection value.
    constexpr bool ESU = UCB && ALGO == RL_ALGO_EXPECTED_SARSA;
    // computed lazily (only lanes whose row needs the UCB values pay for the log;
    // in the all-NaN regime no wave does), then reused until the next increments
    double lnt_es = 0.0;
    bool lnt_ok = false;
    auto lnt_cur = [&](unsigned long long t) -> double {
        if (!lnt_ok) { lnt_es = rl_log((double)t); lnt_ok = true; }
        return lnt_es;
    };
    // visit count of (s, i) as the reference's u128 counter: the step-start value
    // (selection) or with this step's increments (expected SARSA's probabilities)
    auto ucount = [&](uint32_t s, uint32_t i, bool with_step) -> uint64_t {
        const uint32_t idx = qi(0u, s, i);
        if constexpr (SPEC) {
            if (p.ucb_pack) {
                const uint32_t w = NL[idx];
                return p.n_base[s * (uint32_t)A + i] + (uint64_t)(w >> 16) + (with_step ? (uint64_t)(w & 0xffffu) : 0ull);
            }
            return p.n_base[s * (uint32_t)A + i] + (uint64_t)NL[idx] + (with_step ? (uint64_t)D16[idx] : 0ull);
        } else {
            return N[idx];
        }
    };
    if constexpr (TRACES) tcnt = active ? p.tcnt[lane] : 0u;
    const PairCache pc{(uint16_t *)(smem + lay.trc), (double *)(smem + lay.trc + align16(lay.trc_cap * (nthr + 2u) * 2u)),
                       lay.trc_cap, nthr, tid};
    // small tables (S*A <= 256: FrozenLake, CliffWalking): the lane's visited-pair set
    // as a bitmap in registers, rebuilt from the list at launch start.  A visit then
    // needs no scan: a new pair is appended, a visited one gets its E += 1 inside the
    // sweep (the same f64 add, before its use), and "first pair of its state" is the
    // state's A bits
    constexpr bool PBITS = PAIRS && RLAMD_COOP_SWEEP && RLAMD_PAIR_BITS &&
                           (ENV == RL_ENV_CLIFF_WALKING || ENV == RL_ENV_FROZEN_LAKE ||
                            ENV == RL_ENV_FROZEN_LAKE_EDITED);
    constexpr int PBW = ENV == RL_ENV_CLIFF_WALKING ? 6 : 8;   // 48*4 / 64*4 pair ids
    // pair pool (small tables): the visited pairs of a wave's 64 lanes as ONE list of
    // items, tag = pair id (8 bits) | lane in wave << 8 | first-of-state << 15, and
    // its E.  A step sweeps the pool 64 items per round, every thread one item (no
    // per-lane list walk, no owner search), and compacts it in place (the items of
    // lanes whose episode ended leave); a new pair contributes from its own lane and
    // joins at the end.  Items [0, trc_cap) in LDS, the rest in HBM at the same index
    // of the wave's lanes' pair rows (p.tlist / p.trace, lane-major, so the wave's
    // rows are one region of 64*S*A >= any pool); the count in p.tcnt[first lane].
    constexpr bool POOL = PAIRS && pair_pool_env(ENV);
    static_assert(!POOL || (PBITS && A == 4), "pair pool: small-table pair bits");
    const uint32_t pw = tid >> 6, plid = tid & 63u;
    const uint64_t plane0 = (uint64_t)blockIdx.x * p.G + (uint64_t)pw * p.lpw;
    const bool pwave = (uint64_t)pw * p.lpw < p.G && plane0 < p.L;   // the wave holds lanes
    uint16_t *const PT = (uint16_t *)(smem + lay.trc) + pw * lay.trc_cap;
    double *const PE = (double *)(smem + lay.trc + align16(lay.trc_cap * (nthr >> 6) * 2u)) + pw * lay.trc_cap;
    uint4 *const PR = (uint4 *)(smem + lay.trc) + pw * lay.trc_cap;   // RLAMD_POOL_REC16: {E lo, E hi, tag, 0}
    uint4 *const LR = (uint4 *)(smem + lay.lrec) + pw * 64u;          // RLAMD_POOL_LREC: {td lo, td hi, pk, 0}
    uint16_t *const HT = p.tlist + plane0 * SA;
    double *const HE = p.trace + plane0 * SA;
    // the LDS part of the wave's pool, item q < trc_cap
    auto pool_tag = [&](uint32_t q) -> uint32_t {
        if constexpr (RLAMD_POOL_REC16) return PR[q].z;
        else return PT[q];
    };
    auto pool_get = [&](uint32_t q, uint32_t &tg, double &e) {
        if constexpr (RLAMD_POOL_REC16) {
            const uint4 r = PR[q];
            tg = r.z;
            e = __longlong_as_double((long long)(((uint64_t)r.y << 32) | r.x));
        } else {
            tg = PT[q];
            e = PE[q];
        }
    };
    auto pool_put = [&](uint32_t q, uint32_t tg, double e) {
        if constexpr (RLAMD_POOL_REC16) {
            const uint64_t b = (uint64_t)__double_as_longlong(e);
            PR[q] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), tg, 0u);
        } else {
            PT[q] = (uint16_t)tg;
            PE[q] = e;
        }
    };
    uint32_t npool = 0;
    uint32_t pbits[PBW];
#pragma unroll
    for (int i = 0; i < PBW; ++i) pbits[i] = 0u;
    auto pbits_word = [&](uint32_t wi) -> uint32_t {
        uint32_t w = opq(pbits[0]);
#pragma unroll
        for (int i = 1; i < PBW; ++i) w = wi == (uint32_t)i ? opq(pbits[i]) : w;
        return w;
    };
    auto pbits_set = [&](uint32_t id) {
#pragma unroll
        for (int i = 0; i < PBW; ++i) pbits[i] |= (id >> 5) == (uint32_t)i ? (1u << (id & 31u)) : 0u;
    };
    if constexpr (PAIRS && !POOL) { if (active) pair_cache_load(p, pc, lane, tcnt); }
    if constexpr (POOL) {
        npool = pwave ? p.tcnt[plane0] : 0u;
        const uint32_t nl = npool < lay.trc_cap ? npool : lay.trc_cap;
        for (uint32_t q = plid; q < nl; q += 64u) pool_put(q, HT[q], HE[q]);
        __syncthreads();
        // every lane's pair bits from the pool (each lane reads every tag: broadcast)
        constexpr uint32_t TB = 8;
        for (uint32_t q0 = 0; q0 < nl; q0 += TB) {
            uint32_t t[TB];
#pragma unroll
            for (uint32_t k = 0; k < TB; ++k) t[k] = pool_tag(q0 + k < nl ? q0 + k : q0);
#pragma unroll
            for (uint32_t k = 0; k < TB; ++k)
                if (q0 + k < nl && ((t[k] >> 8) & 63u) == plid) pbits_set(t[k] & 0xffu);
        }
        for (uint32_t q0 = nl; q0 < npool; q0 += TB) {
            uint32_t t[TB];
#pragma unroll
            for (uint32_t k = 0; k < TB; ++k) t[k] = HT[q0 + k < npool ? q0 + k : q0];
#pragma unroll
            for (uint32_t k = 0; k < TB; ++k)
                if (q0 + k < npool && ((t[k] >> 8) & 63u) == plid) pbits_set(t[k] & 0xffu);
        }
    } else if constexpr (PBITS) {
        static_assert(A == 4, "a state's pair bits sit in one bitmap word");
        if (active)
            for (uint32_t j = 0; j < tcnt; ++j)
                pbits_set((j < pc.cap ? (uint32_t)pc.TRI[pc.ixi(j)] : (uint32_t)p.tlist[pslot(p, j, lane)]) &
                          0x7fffu);
    }

    // the A visible-flag bytes of LDS row s of table tbl, one per action (A <= 6:
    // the row starts at byte A*(tbl*SL + s), at most 2 bytes into its first word,
    // so two words hold it)
    constexpr uint64_t row_mask = 0x0707070707070707ull >> (8 * (8 - A));
    auto row_flags = [&](uint32_t tbl, uint32_t s) -> uint64_t {
        static_assert(A <= 6, "flag rows span at most two LDS words");
        const uint32_t off = qi(tbl, s, 0u), w = off >> 2;
        const uint64_t two = (uint64_t)QF[w] | ((uint64_t)QF[w + 1u] << 32);
        return (two >> ((off & 3u) * 8u)) & row_mask;
    };
    auto flag_nan = [](uint32_t f) -> bool { return (f & QF_NAN) || (f & (QF_PINF | QF_NINF)) == (QF_PINF | QF_NINF); };
    // f64 image of an entry's word (fixed point: exact, |raw| <= 2^51)
    auto val = [&](int64_t raw) -> double {
        if constexpr (FQ) return as_f64((uint64_t)raw);
        else return q_val(raw);
    };
    // QSH: the f64 images of row s; an A == 4 row (32 bytes, 16-aligned) as two
    // 16-byte reads (element-wise, the compiler issued ds_read2_b64: 19 % slower on cfg 2)
    auto qd_row = [&](uint32_t s, double (&v)[A]) {
        if constexpr (A == 4 && RLAMD_QSH == 2) {
            const double2 *r2 = (const double2 *)__builtin_assume_aligned(QD + qi(0, s, 0), 16);
            const double2 x = r2[0], y = r2[1];
            v[0] = x.x; v[1] = x.y; v[2] = y.x; v[3] = y.y;
        } else {
#pragma unroll
            for (int i = 0; i < A; ++i) v[i] = QD[qi(0, s, i)];
        }
    };
    // raw rows of state s: table 0 and (double policy) table 1, read once per use
    auto load_rows = [&](uint32_t s, int64_t (&ra)[A], int64_t (&rb)[A]) {
        if constexpr (BJC) {
            if (!bj_nonterminal(s)) {                 // read-only terminal row: Q_base
                if (p.bj_tconst) {                    // one value per table (KParams)
#pragma unroll
                    for (int i = 0; i < A; ++i) {
                        ra[i] = p.bj_traw[0];
                        rb[i] = P == 2 ? p.bj_traw[1] : 0;
                    }
                    return;
                }
#pragma unroll
                for (int i = 0; i < A; ++i) {
                    ra[i] = p.q_base[s * (uint32_t)A + i];
                    rb[i] = P == 2 ? p.q_base[SA + s * (uint32_t)A + i] : 0;
                }
                return;
            }
        }
#pragma unroll
        for (int i = 0; i < A; ++i) {
            ra[i] = (int64_t)Q[qi(0, s, i)];
            rb[i] = P == 2 ? (int64_t)Q[qi(1, s, i)] : 0;
        }
    };
    // Agent::get_action = selector(Policy::predict(s)) against the step snapshot;
    // UCB counter increments are applied by the caller after a barrier.
    // single-table Q-learning: the selection's argmax and the TD target's max are
    // of the same row s2, so both come from one pass (argmax_max_*) computed for
    // the whole wave before the selection; `pre` is that argmax (-1: none)
    constexpr bool FUSE_MAX = RLAMD_FUSE_MAX && !UCB && P == 1 && ALGO == RL_ALGO_QLEARNING;
    auto select = [&](uint32_t s, const int64_t (&ra)[A], const int64_t (&rb)[A], int32_t pre = -1) -> uint32_t {
        if constexpr (!UCB) {                       // uniform_epsilon_greed.rs:51-66
            // one compare decides both the draw (skipped when eps == 0) and the branch
            bool explore = L.eps != 0.0;
            if (explore) explore = eps_test(L.rng, L.eps);
            if (explore) return uniform_action<A>(L.rng);
            if constexpr (FUSE_MAX) return (uint32_t)pre;
            if constexpr (FQ) {                     // argmax of predict(): (a + b) / 2.0 (double_tabular_policy.rs:31-39)
                double v[A];
#pragma unroll
                for (int i = 0; i < A; ++i) v[i] = P == 2 ? (as_f64(ra[i]) + as_f64(rb[i])) / 2.0 : as_f64(ra[i]);
                return argmax<A>(v);
            } else {                                // argmax on exact raw values (single table)
                return argmax_i64<A>(ra);
            }
        } else {                                    // upper_confidence_bound.rs:29-42
            double u[A], v[A];
            uint64_t n[A];
            const double lnt = ESU ? lnt_cur(T[0]) : rl_log((double)T[0]);
#pragma unroll
            for (int i = 0; i < A; ++i) {
                v[i] = val(ra[i]);
                if constexpr (P == 2) v[i] = (v[i] + val(rb[i])) / 2.0;
                n[i] = ucount(s, (uint32_t)i, false);
            }
            uint32_t need = ucb_known<A>(v, n, p.ucb_c, lnt, u);
            // argmax (utils.rs:1-11) is decided without the unknown (finite) values
            // when u[0] is NaN (it sticks) or some known u is +inf (the first wins);
            // unknown values are finite only while |c| < 2^1020 (ucb_known)
            const bool c_fin = __builtin_fabs(p.ucb_c) < 0x1p1020;
            bool decided = (need & 1u) == 0u && u[0] != u[0];
#pragma unroll
            for (int i = 0; i < A; ++i)
                decided = decided || (c_fin && ((need >> i) & 1u) == 0u && u[i] == __builtin_inf());
            if (need && !decided) ucb_fill<A>(v, n, p.ucb_c, lnt, need, u);
            return argmax<A>(u);
        }
    };
    // the fused reset's selection (RLAMD_LAZY_ROWS, eps-greedy without FUSE_MAX): row
    // s is read only by the lanes that exploit — the draws come first either way, so
    // the stream and the result are select()'s
    auto select_lazy = [&](uint32_t s) -> uint32_t {
        bool explore = L.eps != 0.0;
        if (explore) explore = eps_test(L.rng, L.eps);
        if (explore) return uniform_action<A>(L.rng);
        int64_t ra[A], rb[A];
        load_rows(s, ra, rb);
        if constexpr (FQ) {
            double v[A];
#pragma unroll
            for (int i = 0; i < A; ++i) v[i] = P == 2 ? (as_f64(ra[i]) + as_f64(rb[i])) / 2.0 : as_f64(ra[i]);
            return argmax<A>(v);
        } else {
            return argmax_i64<A>(ra);
        }
    };
    // fixed point: add n contributions summing to `sum` to entry idx.  Sweep form
    // (the table fits the block, PSA <= nthr): thread i settles entry i every step,
    // so the counter add needs no return value.  Owner form: the step's first
    // contributor (old count 0) settles the entry.
    // PACKC: one LDS atomic per contribution — SUM[idx] holds sum * 2^11 + count
    // (KParams::pack_ok: the host proved |sum| * 2^11 + 2047 < 2^63)
    constexpr bool PACKC = PACK && !FQ;
    auto contribute = [&](uint32_t idx, int64_t sum, uint32_t n) -> bool {
        if constexpr (PACKC) {
            const unsigned long long v = (unsigned long long)(sum * 2048) + n;
            if (sweep) { atomicAdd(&SUM[idx], v); return false; }
            return (atomicAdd(&SUM[idx], v) & 2047ull) == 0ull;
        }
        const uint32_t sh = (idx & 1u) * 16u;
        bool first = false;
        if (sweep) atomicAdd(&CNT[idx >> 1], n << sh);
        else first = ((atomicAdd(&CNT[idx >> 1], n << sh) >> sh) & 0xffffu) == 0u;
        if (sum) atomicAdd(&SUM[idx], (unsigned long long)sum);
        return first;
    };
    // fixed point owner: Q[idx] += mean of the step's contributions (proven in
    // range: no clamp), clear accumulators
    auto settle = [&](uint32_t idx) -> double {
        const int64_t packed = (int64_t)SUM[idx];
        const unsigned long long qold = Q[idx];   // issued beside the SUM read, not after 1/n's
        const uint32_t n = PACKC ? (uint32_t)(packed & 2047) : (uint32_t)CNT16[idx];
        const int64_t sum = PACKC ? (packed >> 11) : packed;
        const double rc = RLAMD_SETTLE_RCPN ? rcp_nr(n)
                                            : ((sweep || n < lay.nrcp) ? RCP[n] : 1.0 / (double)n);   // sweep: n <= block size
        // packed: |sum| < 2^51 (pack_proven), so (double)sum is the 1.5*2^52 magic
        const double sd = PACKC ? __longlong_as_double((long long)(0x4338000000000000ull + (uint64_t)sum)) - 0x1.8p52
                                : (double)sum;
        const double y = __builtin_trunc(sd * rc) + 0x1.8p52;   // mean_delta_rcp
        const int64_t md = (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull);
        const unsigned long long q = qold + (unsigned long long)md;
        Q[idx] = q;
        const double v = q_val((int64_t)q);
        if constexpr (QSH) QD[idx] = v;
        SUM[idx] = 0ull;
        if constexpr (!PACKC) CNT16[idx] = 0;
        return v;
    };
    // row summaries (rmx): thread t settles entries 2t, 2t + 1 (half t & 1 of row t >> 1)
    // as settle() does, then the row's (max, argmax) — first maximum, strict > as
    // argmax_max_f64 — from its half and its partner lane's (t ^ 1, same wave)
    auto settle_pair = [&](uint32_t t) {
        const uint32_t j = 2u * t;
        const ulonglong2 sp = *(const ulonglong2 *)__builtin_assume_aligned(&SUM[j], 16);
        const ulonglong2 qp = *(const ulonglong2 *)__builtin_assume_aligned(&Q[j], 16);
        int64_t md[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t packed = (int64_t)(h ? sp.y : sp.x);
            const uint32_t n = PACKC ? (uint32_t)(packed & 2047) : (uint32_t)CNT16[j + h];
            const int64_t sum = PACKC ? (packed >> 11) : packed;
            const double sd = PACKC ? __longlong_as_double((long long)(0x4338000000000000ull + (uint64_t)sum)) - 0x1.8p52
                                    : (double)sum;
            const double rc = RLAMD_SETTLE_RCPN ? rcp_nr(n) : RCP[n];
            const double y = __builtin_trunc(sd * rc) + 0x1.8p52;
            md[h] = (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull);
        }
        const unsigned long long q0 = qp.x + (unsigned long long)md[0], q1 = qp.y + (unsigned long long)md[1];
        *(ulonglong2 *)__builtin_assume_aligned(&Q[j], 16) = make_ulonglong2(q0, q1);
        const double v0 = q_val((int64_t)q0), v1 = q_val((int64_t)q1);
        *(double2 *)__builtin_assume_aligned(&QD[j], 16) = make_double2(v0, v1);
        *(ulonglong2 *)__builtin_assume_aligned(&SUM[j], 16) = make_ulonglong2(0ull, 0ull);
        if constexpr (!PACKC) *(uint32_t *)&CNT16[j] = 0u;
        const bool up = v1 > v0;
        const double m = up ? v1 : v0;
        const uint32_t a = (t & 1u) * 2u + (up ? 1u : 0u);
        // the partner half (lanes t, t ^ 1): quad_perm [1,0,3,2]
        const uint64_t mb = f64_bits(m);
        const uint32_t pml = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)mb, 0xB1, 0xF, 0xF, false);
        const uint32_t pmh = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(mb >> 32), 0xB1, 0xF, 0xF, false);
        const uint32_t pa = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, 0xB1, 0xF, 0xF, false);
        const double pm = as_f64(((uint64_t)pmh << 32) | pml);
        if ((t & 1u) == 0u) {                 // low half: its entries come first (ties stay)
            const bool hi = pm > m;
            RM[t >> 1] = make_double2(hi ? pm : m, as_f64((uint64_t)(hi ? pa : a)));
        }
    };
    // RLAMD_SETTLE_QUAD: thread t settles entry t (row t >> 2 is one lane quad) and
    // the row summary comes from two DPP combines (pairs, then pairs of pairs; the
    // lower entries win ties, as argmax_max_f64's strict >)
    auto settle_quad = [&](uint32_t t) {
        double m = settle(t);
        uint32_t a = t & 3u;
        auto combine = [&](auto dpp_ctrl_tag, uint32_t bit) {
            constexpr int C = decltype(dpp_ctrl_tag)::value;
            const uint64_t mb = f64_bits(m);
            const uint32_t pl = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)mb, C, 0xF, 0xF, false);
            const uint32_t ph = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(mb >> 32), C, 0xF, 0xF, false);
            const uint32_t pa = (uint32_t)__builtin_amdgcn_mov_dpp((int)a, C, 0xF, 0xF, false);
            const double pm = as_f64(((uint64_t)ph << 32) | pl);
            const bool mine_lo = (t & bit) == 0u;
            const double lo = mine_lo ? m : pm, hi = mine_lo ? pm : m;
            const uint32_t la = mine_lo ? a : pa, ha = mine_lo ? pa : a;
            const bool up = hi > lo;
            m = up ? hi : lo;
            a = up ? ha : la;
        };
        combine(std::integral_constant<int, 0xB1>{}, 1u);   // quad_perm [1,0,3,2]
        combine(std::integral_constant<int, 0x4E>{}, 2u);   // quad_perm [2,3,0,1]
        if ((t & 3u) == 0u) RM[t >> 2] = make_double2(m, as_f64((uint64_t)a));
    };
    // f64 owner: the entry moves by the mean of the step's contributions on their
    // grid (or by the IEEE result of its non-finite ones), NaN canonical
    auto settle_fq = [&](uint32_t idx) {
        const uint32_t w = W[idx], n = w & 0xfffu;
        const uint32_t f = w >> 28;
        if (n == 0u && f == 0u) return;            // sweep form: untouched this step
        double dl;
        if (f) {
            dl = nf_value(f);
        } else {
            const double rc = (sweep || n < lay.nrcp) ? RCP[n] : 1.0 / (double)n;
            dl = __builtin_ldexp((double)(int64_t)SUM[idx] * rc, fq_grid(((w >> 16) & 0xfffu) - 1u));
        }
        const double q = canon_nan(as_f64(Q[idx]) + dl);
        Q[idx] = f64_bits(q);
        SUM[idx] = 0ull;
        W[idx] = 0u;
        if constexpr (SPEC) QF8[idx] = (uint8_t)value_flags(q);
    };
    // traces: every action of a visited state receives a contribution
    // (elegibility_traces_agent.rs:82-96), so the A entries of an LDS row share
    // one count n — one counter per (table, row) in the CNT region (u32 words):
    // one atomic per visited state instead of A.  Row sweep when every row has a
    // thread, else the first contributor of a row lists it.
    uint32_t *const CNTR = CNT;
    // row sweep: every row settled by a strided pass (rows with no count return at
    // once), so a visit's count needs no return value.  Pair pools (small tables,
    // P * S <= 128 rows) always sweep: the list form's returning atomic made every
    // first-of-state item wait for all of the wave's outstanding LDS operations
    const bool rsweep = POOL || (uint32_t)P * SL <= nthr;
    auto qi_row = [&](uint32_t tbl, uint32_t row, uint32_t a) -> uint32_t {
        return LDS_AM ? tbl * SAL + a * SL + row : tbl * SAL + row * (uint32_t)A + a;
    };
    // f64 traces: one grid per group step, 2^e with e from the step's largest finite
    // |td| and the trace bound (oracle rlref.c fq_step_combine)
    auto contrib_tr = [&](uint32_t idx, double d, int e) {
        if (__builtin_isfinite(d)) {
            // |raw| < 2^51 (trace_grid_k's guard bits): rint and the int64 conversion
            // in one magic add (fq_raw's general conversion was 5 f64 operations)
            const double y = __builtin_ldexp(d, -e) + 0x1.8p52;
            const int64_t raw = (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull);
            if (raw) atomicAdd(&SUM[idx], (unsigned long long)raw);
        } else {
            atomicOr(&SFLW[idx >> 2], (nf_flag(d) << SFL_SH) << ((idx & 3u) * 8u));
        }
    };
    auto settle_row = [&](uint32_t rid, int e) {   // rid = tbl*SL + LDS row
        const uint32_t n = CNTR[rid];
        if (n == 0u) return;
        const double rc = n < lay.nrcp ? RCP[n] : 1.0 / (double)n;
        const uint32_t tbl = rid / SL, row = rid - tbl * SL;
#pragma unroll
        for (int b = 0; b < A; ++b) {
            const uint32_t idx = qi_row(tbl, row, (uint32_t)b);
            const uint32_t f = ((uint32_t)SFL8[idx] >> SFL_SH) & QF_MASK;
            const double dl = f ? nf_value(f) : __builtin_ldexp((double)(int64_t)SUM[idx] * rc, e);
            const double q = canon_nan(as_f64(Q[idx]) + dl);
            Q[idx] = f64_bits(q);
            SUM[idx] = 0ull;
            if constexpr (SPEC) QF8[idx] = (uint8_t)value_flags(q);
            else if (f) SFL8[idx] = 0;
        }
        CNTR[rid] = 0u;
    };
    // wave-level per-launch counters (scalar registers: ballot popcounts)
    uint32_t c_train = 0, c_eval = 0, c_tep = 0, c_eep = 0;
    unsigned long long *const RSUM = &ACC[4];
    // RLAMD_RSUM_REG: this lane's finished training episodes' rint(reward * 2^16),
    // summed in registers (int64 adds are exact and order free)
    int64_t rsum_lane = 0;

    // FrozenLake family, one action per step (no reset-and-step): the step's table
    // word trans[(s, a)] is read a step ahead (after the previous selection)
    constexpr bool TRPF = RLAMD_TRPF && RS == 0 &&
                          (ENV == RL_ENV_FROZEN_LAKE || ENV == RL_ENV_FROZEN_LAKE_EDITED);
    uint32_t wpf = 0;
    if constexpr (TRPF) wpf = tabs.trans[tidx<LDS_AM, 4>(tabs, L.s, L.a)];
    // Taxi: the transition word of the lane's (s, a) from the host's table (HBM, 12 KB:
    // L2-resident), read one step ahead — after the selection that fixes the next
    // step's action — instead of decoding / encoding the state (rl_taxi.h taxi_word,
    // which the host checked equal to the table); not with the reset-and-step schedule
    constexpr bool TXPF = RLAMD_TAXI_PF && ENV == RL_ENV_TAXI && (UCB || RS == 0);
    uint32_t wtx = 0;
    if constexpr (TXPF) wtx = p.trans[(L.s < S ? L.s : 0u) * (uint32_t)A + (L.a < (uint32_t)A ? L.a : 0u)];
    // reset-and-step in effect (uniform over the block)
    const bool rs_on = (!UCB && RS != 0) && (RS == 1 || p.reset_step);
    for (uint32_t k = 0; k < p.K; ++k) {
        // ---------------- one synchronous step: each live lane either RESETs
        // (env.reset() + get_action, src/agent.rs:83-84) or STEPs (env.step +
        // get_action + update, :88-97); one selection per lane per step.
        const bool alive = L.mode != RL_MODE_DONE;
        bool doR = alive && L.need_reset;
        bool doS = alive && !L.need_reset;
        const uint32_t mode_before = L.mode;
        uint32_t s2 = 0, a2 = 0;
        double r = 0.0;
        bool term = false;
        int64_t ra2[A], rb2[A];
        // reset-and-step schedule (KParams::reset_step, eps-greedy only): a lane
        // that needs a reset does env.reset() + get_action against the step
        // snapshot and then steps in the same synchronous step
        bool fused = false;
        if constexpr (!UCB && RS != 0) {   // RS: the schedule as a compile-time constant (-1: KParams)
            if (RS == 1 || p.reset_step) {
                if (doR && RLAMD_LAZY_ROWS && !FUSE_MAX) {
                    const uint32_t s0 = E::reset(L.z, L.rng, tabs);
                    L.ready = true;
                    L.a = select_lazy(s0);
                    L.s = s0;
                    L.need_reset = false;
                    L.epi_reward = 0.0;
                    L.epi_len = 0;
                    fused = true;
                } else if (doR) {
                    const uint32_t s0 = E::reset(L.z, L.rng, tabs);
                    L.ready = true;
                    load_rows(s0, ra2, rb2);
                    int32_t pre = -1;
                    if constexpr (FUSE_MAX) {
                        if constexpr (FQ) {
                            double v[A], m;
#pragma unroll
                            for (int i = 0; i < A; ++i) v[i] = as_f64(ra2[i]);
                            pre = (int32_t)argmax_max_f64<A>(v, m);
                        } else if constexpr (QSH) {
                            if (rmx) {
                                pre = (int32_t)(uint32_t)f64_bits(RM[s0].y);
                            } else {
                                double v[A], m;
                                qd_row(s0, v);
                                pre = (int32_t)argmax_max_f64<A>(v, m);
                            }
                        } else {
                            pre = (int32_t)argmax_i64<A>(ra2);
                        }
                    }
                    L.a = select(s0, ra2, rb2, pre);
                    L.s = s0;
                    L.need_reset = false;
                    L.epi_reward = 0.0;
                    L.epi_len = 0;
                    fused = true;
                }
                doR = false;
                doS = alive;
            }
        }
        if constexpr (ENV == RL_ENV_FROZEN_LAKE || ENV == RL_ENV_FROZEN_LAKE_EDITED) {
            uint32_t pos = L.s;                    // reset or step in one predicated block
            const uint32_t w = TRPF ? wpf : tabs.trans[tidx<LDS_AM, 4>(tabs, L.s, L.a)];
            fl_advance<ENV == RL_ENV_FROZEN_LAKE_EDITED, SLIP, LDS_AM>(doR, doS, pos, L.z, w, L.rng, tabs, s2, r,
                                                                       term);
            L.ready = doR ? true : (term ? false : L.ready);
        } else if constexpr (ENV == RL_ENV_BLACKJACK && RLAMD_BJ_ONE_LOOP) {
            E::advance(doR, doS, L.z, L.a, L.rng, s2, r, term);
            L.ready = doR ? true : (doS && term ? false : L.ready);
        } else if (doR) {
            s2 = E::reset(L.z, L.rng, tabs);
            L.ready = true;
        } else if (doS) {
            uint32_t pos = L.s;
            if constexpr (TXPF) E::step_word(L.z, wtx, tabs, s2, r, term);
            else E::template step<SLIP, LDS_AM>(pos, L.z, L.a, L.rng, tabs, s2, r, term);
            if (term) L.ready = false;
        }
        // the previous step's settle (Q, flags, counters) before this step's reads:
        // the env step above touches no shared table, so it overlaps the settle
        // (reset-and-step reads Q for its reset lanes' selection: barrier at the end of the step)
        if (RLAMD_LATE_B3 && k > 0 && !rs_on) __syncthreads();
        // UCB + expected SARSA (SPEC): the visible flags of row s2 decide most of
        // the step without Q values or counters (the regime is mostly
        // non-finite rows).  u_0 NaN sticks as the argmax (utils.rs:1-11); any
        // non-finite value in the target row makes some u_i non-finite (v_i, or
        // v_i + b0 when n_i = 0: inf or NaN either way), so sum(u) is non-finite,
        // some p_i is NaN and the expectation — and td — are NaN
        // (upper_confidence_bound.rs:48-63, src/agent.rs:35-45).
        bool sel_nan0 = false, tgt_nf = false;
        if constexpr (SPEC) {
            const uint64_t f0 = row_flags(0u, s2), f1 = P == 2 ? row_flags(1u, s2) : 0ull;
            sel_nan0 = flag_nan((uint32_t)f0 & 0xffu) || (P == 2 && flag_nan((uint32_t)f1 & 0xffu));
            tgt_nf = ((((P == 2 && !L.dflag) ? f1 : f0) & row_mask) != 0ull);
        }
        const bool train_lane = doS && L.mode == RL_MODE_TRAIN;
        if constexpr (RLAMD_EARLY_COUNT) {
            // the step's counters from masks formed here (L.mode changes only in the
            // bookkeeping): counted at the end, the flags crossed the step's branches
            // and barriers and each ballot re-materialised its mask (2 VALU each)
            c_train += (uint32_t)__popcll(__ballot(train_lane));
            c_tep += (uint32_t)__popcll(__ballot(train_lane && term));
            if (EPI > 0 || (EPI < 0 && p.episodic)) {
                const bool ev_lane = doS && L.mode == RL_MODE_EVAL;
                c_eval += (uint32_t)__popcll(__ballot(ev_lane));
                c_eep += (uint32_t)__popcll(__ballot(ev_lane && term));
            }
        }
        if (!SPEC || !(sel_nan0 && (tgt_nf || !train_lane))) load_rows(s2, ra2, rb2);   // s2 == 0 on idle lanes
        else {
#pragma unroll
            for (int i = 0; i < A; ++i) ra2[i] = rb2[i] = 0;
        }
        // RLAMD_QA_EARLY2: the TD's Q(s, a) word (table vt) read with the target rows,
        // its latency under the selection (L.s, L.a, L.dflag are final here, also
        // after a fused reset)
        int64_t qa_raw_pre = 0;
        constexpr bool QAE2 = RLAMD_QA_EARLY2 && TRACES && !QSH && !SPEC;
        if constexpr (QAE2) {
            if (BJC && !bj_nonterminal(L.s)) qa_raw_pre = 0;   // never a TD source (terminal rows are not stepped from)
            else qa_raw_pre = (int64_t)Q[qi((P == 2 && !L.dflag) ? 1u : 0u, L.s, L.a)];
        }
        uint32_t rm_pad = 0;                // rmx: the row summary's 4th dword (see below)
        double qa_pre = 0.0;                // rmx: Q(s, a) read early
        int64_t rmax = 0;                   // FUSE_MAX: utils::max of row s2 (the Q-learning target)
        double rmaxd = 0.0;
        int32_t rarg = -1;
        if constexpr (FUSE_MAX) {
            if constexpr (FQ) {
                double v[A];
#pragma unroll
                for (int i = 0; i < A; ++i) v[i] = as_f64(ra2[i]);
                rarg = (int32_t)argmax_max_f64<A>(v, rmaxd);
                if constexpr (RLAMD_FUSE_MAX == 2) asm volatile("" : "+v"(rarg), "+v"(rmaxd));
            } else if constexpr (QSH) {
                if (rmx) {
                    // no pin: the load's wait can sink to the first use (the exploit
                    // branch, the TD), past the eps test and the exploring draw.  Its
                    // unused 4th dword is kept live up to the TD (rm_pad): else the
                    // compiler reuses that register at once and must wait for the load
                    const double2 rm = RM[s2];
                    rmaxd = rm.x;
                    rarg = (int32_t)(uint32_t)f64_bits(rm.y);
                    rm_pad = (uint32_t)(f64_bits(rm.y) >> 32);
                    // Q(s, a) of the TD, read with the summary (one action per step:
                    // (s, a) is known since the last step; RLAMD_QA_EARLY)
                    if (RLAMD_QA_EARLY && !rs_on) qa_pre = QD[qi(0u, L.s, L.a)];
                    if constexpr (RLAMD_RM_PIN) asm volatile("" : "+v"(rarg), "+v"(rmaxd));
                } else {
                    double v[A];
                    qd_row(s2, v);
                    rarg = (int32_t)argmax_max_f64<A>(v, rmaxd);
                    if constexpr (RLAMD_FUSE_MAX == 2) asm volatile("" : "+v"(rarg), "+v"(rmaxd));
                }
            } else {
                rarg = (int32_t)argmax_max_i64<A>(ra2, rmax);
                // pin both here (empty asm): left alone, the compiler sinks the index into
                // the exploit branch and the max into the TD branch, redoing the compares
                if constexpr (RLAMD_FUSE_MAX == 2) asm volatile("" : "+v"(rarg), "+v"(rmax));
            }
        }
        if (alive) a2 = sel_nan0 ? 0u : select(s2, ra2, rb2, rarg);
        // the next step's table word (s2, a2) read now: the table is constant, and
        // the read's latency then overlaps the update and its barriers
        if constexpr (TRPF) wpf = tabs.trans[tidx<LDS_AM, 4>(tabs, s2, a2)];
        if constexpr (TXPF) wtx = p.trans[s2 * (uint32_t)A + a2];
        uint32_t d_own = 0xffffffffu;   // SPEC: the step-count entry this lane folds at step end
        if constexpr (SPEC) {
            // the step's increments go to the step counts / T[1], apart from what this
            // step's selections read (launch counts, T[0]), so no barrier separates the
            // two; expected SARSA's probabilities read both after the arrival below
            if (alive) {
                const uint32_t idx = qi(0, s2, a2);
                if (p.ucb_pack) {
                    if ((atomicAdd(&NL[idx], 1u) & 0xffffu) == 0u) d_own = idx;
                } else {
                    const uint32_t sh = (idx & 1u) * 16u;
                    if (((atomicAdd(&D32[idx >> 1], 1u << sh) >> sh) & 0xffffu) == 0u) d_own = idx;
                }
            }
            const uint32_t c = (uint32_t)__popcll(__ballot(alive));
            if ((tid & 63u) == 0 && c) atomicAdd(&T[1], (unsigned long long)c);
            // one-sided barrier: every wave announces that its increments are in
            // (ARR counts arrivals over the launch); only a wave with a lane whose
            // target row is finite reads the counts / T, so only such a wave waits for
            // all arrivals of this step.  No wave passes the end-of-step barrier before
            // arriving, so ARR >= (k+1) * waves means exactly that.  In the all-NaN
            // regime no wave waits.  What the others go on to do meanwhile (their
            // contributions) is invisible to the step's readers.
            uint32_t *ARR = (uint32_t *)(T + 2);
            __threadfence_block();
            if ((tid & 63u) == 0) atomicAdd(ARR, 1u);
            if (__ballot(train_lane && !tgt_nf)) {
                const uint32_t goal = (k + 1u) * (nthr >> 6);
                while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ARR, __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_WORKGROUP)) < goal)
                    __builtin_amdgcn_s_sleep(1);
                __threadfence_block();
            }
            lnt_ok = false;   // this step's probabilities and the next selection use ln(T_{k+1})
        } else if constexpr (UCB) {
            __syncthreads();
            if (alive) atomicAdd(&N[qi(0, s2, a2)], 1ull);
            const uint32_t c = (uint32_t)__popcll(__ballot(alive));
            if ((tid & 63u) == 0 && c) atomicAdd(&T[0], (unsigned long long)c);
            // the next reader is the next step's selection, after the end-of-step barrier
        }
        // ---------------- update (one_step_agent.rs:53-86 / elegibility_traces_agent.rs:61-104)
        // Contributions go to SUM/CNT, never to Q, so no barrier is needed before them.
        // throughput mode (EPI 0): rl_agent_run leaves every live lane in TRAIN mode
        // (no eval interleave, no target: after_step<0> never changes a mode)
        const bool train = (EPI == 0 && RLAMD_RUN_TRAIN) ? doS : (doS && L.mode == RL_MODE_TRAIN);
        const uint32_t vt = (P == 2 && !L.dflag) ? 1u : 0u;   // get_values: flag ? alpha : beta
        const uint32_t ut = (P == 2 && L.dflag) ? 1u : 0u;    // update:     flag ? beta : alpha
        double td = 0.0;
        if (train) {
            int64_t rv[A];
#pragma unroll
            for (int i = 0; i < A; ++i) rv[i] = vt ? rb2[i] : ra2[i];
            double fq;
            if constexpr (ALGO == RL_ALGO_QLEARNING && !SPEC) {
                if constexpr (FQ) {
                    if constexpr (FUSE_MAX) {
                        fq = rmaxd;
                    } else {
                        double v[A];
#pragma unroll
                        for (int i = 0; i < A; ++i) v[i] = as_f64(rv[i]);
                        fq = vmax<A>(v);                   // utils::max
                    }
                } else if constexpr (QSH) {
                    fq = rmaxd;                            // the f64 image's max (exact)
                } else {
                    fq = q_val(FUSE_MAX ? rmax : max_i64<A>(rv));   // utils::max on exact images
                }
            } else if constexpr (ALGO == RL_ALGO_SARSA && !SPEC) {
                fq = val(pick<A>(rv, a2));
            } else if (SPEC && tgt_nf) {
                fq = __builtin_nan("");
            } else {
                double q2[A], pr[A];
#pragma unroll
                for (int i = 0; i < A; ++i) q2[i] = val(rv[i]);
                if constexpr (!UCB) {
                    eps_probs<A>(L.eps, q2, pr);
                } else {                                   // upper_confidence_bound.rs:48-63
                    const double lnt = lnt_cur(T[0] + T[1]);
                    uint64_t n[A];
#pragma unroll
                    for (int i = 0; i < A; ++i) n[i] = ucount(s2, (uint32_t)i, true);
                    uint32_t need = ucb_known<A>(q2, n, p.ucb_c, lnt, pr);
                    // a known non-finite u makes the sum non-finite, so some p_i is
                    // inf/inf or NaN and the expectation is NaN: skip the rest
                    bool nan_fq = false;
#pragma unroll
                    for (int i = 0; i < A; ++i) nan_fq = nan_fq || (((need >> i) & 1u) == 0u && !__builtin_isfinite(pr[i]));
                    if (!nan_fq) {
                        if (need) ucb_fill<A>(q2, n, p.ucb_c, lnt, need, pr);
                        double sum = 0.0;
#pragma unroll
                        for (int i = 0; i < A; ++i) sum += pr[i];
#pragma unroll
                        for (int i = 0; i < A; ++i) pr[i] /= sum;
                    } else {
#pragma unroll
                        for (int i = 0; i < A; ++i) pr[i] = __builtin_nan("");
                    }
                }
                fq = future_q<ALGO, A>(q2, a2, pr);
            }
            if (SPEC && tgt_nf) {
                td = __builtin_nan("");                    // r + gamma * NaN - q
            } else {
                const uint32_t qidx = qi(vt, L.s, L.a);
                const double qa = QSH ? ((RLAMD_QA_EARLY && rmx && !rs_on) ? qa_pre : QD[qidx])
                                      : val(QAE2 ? qa_raw_pre : (int64_t)Q[qidx]);
                td = r + p.gamma * fq - qa;
                if constexpr (QSH && !RLAMD_RM_PIN) asm volatile("" ::"v"(rm_pad));
            }
        }
        if constexpr (!TRACES) {
            const uint32_t idx = qi(ut, L.s, L.a);
            if constexpr (FQ) {
                // pass 1: the step's largest code per entry (+1: 0 marks an untouched
                // entry) or the kinds of its non-finite contributions, in the top bits
                // (a max after them leaves them: the code no longer matters then); the
                // first contributor owns the entry's settle
                double d = 0.0;
                bool fin = true, owner = false;
                if (train) {
                    d = p.lr * td;                         // tabular_policy.rs:36 (lr * td)
                    fin = __builtin_isfinite(d);
                    const uint32_t old = fin ? atomicMax(&W[idx], (f64_code(d) + 1u) << 16)
                                             : atomicOr(&W[idx], nf_flag(d) << 28);
                    owner = old == 0u;
                }
                __syncthreads();   // every code in
                // pass 2: the contribution on its entry's grid, and the count — only
                // where every contribution was finite: an entry with non-finite kinds
                // moves by their IEEE sum, which needs neither (settle_fq)
                if (train && (RLAMD_NF_SKIP == 0 || fin)) {
                    const uint32_t w = W[idx];
                    if (fin && (w >> 28) == 0u) {
                        const int64_t raw = fq_raw(d, fq_grid(((w >> 16) & 0xfffu) - 1u));
                        if (raw) atomicAdd(&SUM[idx], (unsigned long long)raw);
                        if (RLAMD_NF_SKIP) atomicAdd(&W[idx], 1u);
                    }
                    if (!RLAMD_NF_SKIP) atomicAdd(&W[idx], 1u);
                }
                __syncthreads();   // all contributions in, all Q reads done
                if (sweep) { if (tid < PSAL) settle_fq(tid); }
                else if (owner) settle_fq(idx);
            } else {
                bool owner = false;
                if (train) owner = contribute(idx, rint_i64_small(p.lr40 * td), 1u);   // q_fix_inrange(lr * td)
                __syncthreads();   // all contributions in, all Q reads done
                if (rmx) {
                    if constexpr (RLAMD_SETTLE_QUAD) { if (tid < PSAL) settle_quad(tid); }
                    else { if (tid < PSAL / 2u) settle_pair(tid); }
                }
                else if (sweep) { if (tid < PSAL) settle(tid); }
                else if (owner) settle(idx);
            }
        } else {
            // accumulating trace: E[s][a] += 1, then for every visited (o, b):
            // Q[o][b] += lr*(td*E[o][b]); E[o][b] *= gamma*lambda; E cleared on
            // termination (elegibility_traces_agent.rs:75-101).
            // The group step's grid: 2^e from the largest finite |td| of its lanes
            int e_tr;
            {
                const uint32_t c = (train && __builtin_isfinite(td)) ? f64_code(td) : 0u;
                const uint32_t wm = wave_max_u32(c);
                if ((tid & 63u) == 0 && wm) atomicMax(GCODE, wm);
                __syncthreads();
                e_tr = fq_grid(GCODE[0]) + p.trace_k;
            }
            // a visited state's row count n += 1 (settle_row's mean)
            auto row_hit = [&](uint32_t rid) {
                if (rsweep) atomicAdd(&CNTR[rid], 1u);
                else if (atomicAdd(&CNTR[rid], 1u) == 0u) LIST[atomicAdd(&LISTN[0], 1u)] = (uint16_t)rid;
            };
            if constexpr (POOL) {
                // this lane's visit: a visited pair gets its E += 1 inside the sweep (hid);
                // a new pair contributes below with E = 1 and then joins the pool
                uint32_t hid = 0x1ffu, nid = 0u;
                bool newp = false, first_new = false;
                if (train) {
                    const uint32_t id = L.s * (uint32_t)A + L.a;
                    const uint32_t w = pbits_word(id >> 5);
                    if ((w >> (id & 31u)) & 1u) {
                        hid = id;
                    } else {
                        newp = true;
                        nid = id;
                        first_new = ((w >> ((L.s * (uint32_t)A) & 31u)) & 0xfu) == 0u;
                        pbits_set(id);
                    }
                }
                // shuffled to the lane's items with its td: the E += 1 pair (bits 0-8),
                // the update table (16), "trains this step" (20), "its episode ends" (21)
                const uint32_t pk = hid | (ut << 16) | (train ? 1u << 20 : 0u) | (train && term ? 1u << 21 : 0u);
                const uint32_t C = lay.trc_cap;
                uint32_t wpos = 0;                             // items kept so far (uniform)
                constexpr uint32_t U = RLAMD_SWEEP_U;
                if constexpr (RLAMD_POOL_LREC) {
                    // the lane's {td, pk} for its items (same wave: LDS operations of a
                    // wave complete in order, so no barrier between the write and the reads)
                    const uint64_t tb = (uint64_t)__double_as_longlong(td);
                    LR[plid] = make_uint4((uint32_t)tb, (uint32_t)(tb >> 32), pk, 0u);
                    __builtin_amdgcn_wave_barrier();
                }
                for (uint32_t q0 = 0; q0 < npool; q0 += 64u * U) {
                    uint32_t tg[U], pkv[U];
                    double ev[U], tdv[U];
                    // items past the LDS part only in a wave-uniform slow path (a per-item
                    // select let the compiler load both copies of every item)
                    if (q0 + 64u * U <= C) {
#pragma unroll
                        for (uint32_t u = 0; u < U; ++u) {
                            const uint32_t q = q0 + 64u * u + plid;
                            pool_get(q < npool ? q : 0u, tg[u], ev[u]);
                        }
                    } else {
#pragma unroll
                        for (uint32_t u = 0; u < U; ++u) {
                            const uint32_t q = q0 + 64u * u + plid;
                            tg[u] = 0u;
                            ev[u] = 0.0;
                            if (q < npool) {
                                if (q < C) pool_get(q, tg[u], ev[u]);
                                else { tg[u] = HT[q]; ev[u] = HE[q]; }
                            }
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        const uint32_t il = (tg[u] >> 8) & 63u;
                        if constexpr (RLAMD_POOL_LREC) {
                            const uint4 r = LR[il];
                            tdv[u] = __longlong_as_double((long long)(((uint64_t)r.y << 32) | r.x));
                            pkv[u] = r.z;
                        } else {
                            tdv[u] = __shfl(td, (int)il, 64);
                            pkv[u] = (uint32_t)__shfl((int)pk, (int)il, 64);
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        const uint32_t q = q0 + 64u * u + plid;
                        const bool valid = q < npool;
                        const bool istr = valid && ((pkv[u] >> 20) & 1u);
                        const bool keep = valid && !((pkv[u] >> 21) & 1u);
                        double en = ev[u];
                        if constexpr (RLAMD_POOL_BF) {
                            // branch-free: every valid item adds its contribution and its
                            // row count — 0 for the items of lanes that do not train this
                            // step (integer adds of 0 change nothing)
                            const uint32_t id = tg[u] & 0xffu, uto = P == 2 ? (pkv[u] >> 16) & 1u : 0u;
                            const double e1 = id == (pkv[u] & 0x1ffu) ? ev[u] + 1.0 : ev[u];
                            const uint32_t o = id >> 2, b = id & 3u;   // A == 4
                            const bool first = istr && (tg[u] & 0x8000u);
                            const double d = p.lr * (tdv[u] * e1);
                            const bool fin = __builtin_isfinite(d);
                            // |raw| < 2^51 for finite d (trace_grid_k's guard bits): the magic add
                            const double y = __builtin_ldexp(d, -e_tr) + 0x1.8p52;
                            const int64_t raw = (istr && fin)
                                ? (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull) : (int64_t)0;
                            if (valid) {
                                atomicAdd(&SUM[qi(uto, o, b)], (unsigned long long)raw);
                                atomicAdd(&CNTR[uto * SL + lrow(o)], first ? 1u : 0u);
                            }
                            trace_states += first ? 1u : 0u;
                            if (__builtin_expect(__ballot(istr && !fin) != 0ull, 0)) {   // rare: non-finite kinds
                                if (istr && !fin) contrib_tr(qi(uto, o, b), d, e_tr);
                            }
                            en = istr ? e1 * p.gl : ev[u];
                        } else if (istr) {
                            const uint32_t id = tg[u] & 0xffu, uto = P == 2 ? (pkv[u] >> 16) & 1u : 0u;
                            const double e1 = id == (pkv[u] & 0x1ffu) ? ev[u] + 1.0 : ev[u];
                            const uint32_t o = id >> 2, b = id & 3u;   // A == 4
                            if (tg[u] & 0x8000u) {
                                ++trace_states;
                                row_hit(uto * SL + lrow(o));
                            }
                            contrib_tr(qi(uto, o, b), p.lr * (tdv[u] * e1), e_tr);
                            en = e1 * p.gl;
                        }
                        const uint64_t m = __ballot(keep);
                        const uint32_t pos = wpos + lanes_below(m);
                        if (RLAMD_POOL_BF && wpos + 64u <= C) {   // uniform: the round's kept items fit in LDS
                            if (keep) pool_put(pos, tg[u], en);
                        } else if (keep) {
                            if (wpos + 64u <= C || pos < C) pool_put(pos, tg[u], en);
                            else { HT[pos] = (uint16_t)tg[u]; HE[pos] = en; }
                        }
                        wpos += (uint32_t)__popcll(m);
                    }
                }
                if (newp) {
                    if (first_new) {
                        ++trace_states;
                        row_hit(ut * SL + lrow(L.s));
                    }
                    contrib_tr(qi(ut, L.s, L.a), p.lr * (td * 1.0), e_tr);
                }
                const bool keepn = newp && !term;
                const uint64_t m = __ballot(keepn);
                if (keepn) {
                    const uint32_t pos = wpos + lanes_below(m);
                    const uint16_t tag = (uint16_t)(nid | (plid << 8) | (first_new ? 0x8000u : 0u));
                    const double en = 1.0 * p.gl;
                    if (pos < C) pool_put(pos, tag, en);
                    else { HT[pos] = tag; HE[pos] = en; }
                }
                npool = wpos + (uint32_t)__popcll(m);
            } else if constexpr (PAIRS && RLAMD_COOP_SWEEP) {
                uint32_t hid = 0xffffu;      // PBITS: the visited pair whose E += 1 the sweep applies
                if constexpr (PBITS) {
                    if (train) {
                        const uint32_t id = L.s * (uint32_t)A + L.a;
                        const uint32_t w = pbits_word(id >> 5);
                        if ((w >> (id & 31u)) & 1u) {
                            hid = id;
                        } else {
                            const bool first = ((w >> ((L.s * (uint32_t)A) & 31u)) & 0xfu) == 0u;
                            const uint16_t tag = (uint16_t)(id | (first ? 0x8000u : 0u));
                            const uint32_t j = tcnt++;
                            if (j < pc.cap) {
                                pc.TRI[pc.ixi(j)] = tag;
                                pc.TRE[pc.ixe(j)] = 1.0;
                            } else {
                                p.tlist[pslot(p, j, lane)] = tag;
                                p.trace[pslot(p, j, lane)] = 1.0;
                            }
                            pbits_set(id);
                        }
                    }
                } else {
                    if (train) pair_visit<A>(p, pc, lane, L.s, L.a, tcnt);
                }
                // wave-cooperative sweep: the (lane, slot) items of the wave's 64
                // lanes are dealt out 64 at a time, so a wave takes ceil(sum/64)
                // rounds instead of its longest list (episode lengths are long-tailed)
                const uint32_t lid = tid & 63u, wbase = tid & ~63u;
                const uint32_t npl = train ? tcnt : 0u;
                uint32_t incl = npl;
#pragma unroll
                for (uint32_t o = 1; o < 64; o <<= 1) {
                    const uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
                    if (lid >= o) incl += v;
                }
                const uint32_t excl = incl - npl;
                const uint32_t T = (uint32_t)__shfl((int)incl, 63, 64);
                // RLAMD_SWEEP_U rounds per iteration, every stage interleaved across
                // them (owner searches, gathers, loads, then the updates): with 2
                // waves per SIMD (cfg 4) the rounds' LDS / HBM round trips overlap
                // instead of queueing one dependent chain per round
                constexpr uint32_t U = RLAMD_SWEEP_U;
                const bool nonempty = npl != 0u;
                for (uint32_t q0 = 0; q0 < T; q0 += 64u * U) {
                    uint32_t qv[U], lo[U], exo[U];
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) { qv[u] = q0 + 64u * u + lid; lo[u] = 0; exo[u] = 0; }
#if RLAMD_OWNER_SCAN
                    // owner of item q: the last non-empty lane with excl <= q.  The owner of
                    // q0 from one ballot; then the few non-empty lanes whose lists start inside
                    // this iteration's items, in lane order, by readlane (scalar, no LDS
                    // round trip): a short uniform loop instead of 6 dependent shuffles
                    {
                        const uint32_t qend = q0 + 64u * U - 1u;
                        const uint64_t m0 = __ballot(nonempty && excl <= q0);
                        const uint32_t own0 = 63u - (uint32_t)__builtin_clzll(m0);   // q0 < T: m0 != 0
                        const uint32_t ex0 = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)own0);
#pragma unroll
                        for (uint32_t u = 0; u < U; ++u) { lo[u] = own0; exo[u] = ex0; }
                        uint64_t m = __ballot(nonempty && excl > q0 && excl <= qend);
                        while (m) {
                            const uint32_t jl = (uint32_t)__builtin_ctzll(m);
                            m &= m - 1ull;
                            const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)excl, (int)jl);
#pragma unroll
                            for (uint32_t u = 0; u < U; ++u) {
                                const bool in = e <= qv[u];
                                lo[u] = in ? jl : lo[u];
                                exo[u] = in ? e : exo[u];
                            }
                        }
                    }
#else
#pragma unroll
                    for (uint32_t st = 32; st; st >>= 1) {   // owner: last lane with excl <= q
#pragma unroll
                        for (uint32_t u = 0; u < U; ++u) {
                            const uint32_t e = (uint32_t)__shfl((int)excl, (int)(lo[u] + st), 64);
                            if (e <= qv[u]) lo[u] += st;
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) exo[u] = (uint32_t)__shfl((int)excl, (int)lo[u], 64);
#endif
                    uint32_t jv[U], utv[U], wv[U], colv[U], hidv[U];
                    uint64_t lanev[U];
                    double tdv[U], evv[U];
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        jv[u] = qv[u] - exo[u];
                        tdv[u] = __shfl(td, (int)lo[u], 64);
                        utv[u] = P == 2 ? (uint32_t)__shfl((int)ut, (int)lo[u], 64) : 0u;
                        hidv[u] = PBITS ? (uint32_t)__shfl((int)hid, (int)lo[u], 64) : 0xffffu;
                        lanev[u] = lane - lid + lo[u];        // lanes of a wave are consecutive
                        colv[u] = wbase + lo[u];   // the owner's thread: its slot column
                    }
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        wv[u] = 0; evv[u] = 0.0;
                        if (qv[u] < T) {
                            const bool in_lds = jv[u] < pc.cap;
                            wv[u] = in_lds ? (uint32_t)pc.TRI[pc.ixi_t(jv[u], colv[u])] : (uint32_t)p.tlist[pslot(p, jv[u], lanev[u])];
                            evv[u] = in_lds ? pc.TRE[pc.ixe_t(jv[u], colv[u])] : p.trace[pslot(p, jv[u], lanev[u])];
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < U; ++u) {
                        if (qv[u] < T) {
                            const uint32_t w = wv[u], j = jv[u], col = colv[u], ut_o = utv[u];
                            const uint32_t id = w & 0x7fffu;
                            const double ev = (PBITS && id == hidv[u]) ? evv[u] + 1.0 : evv[u], td_o = tdv[u];
                            const bool in_lds = j < pc.cap;
                            const uint32_t o = id / (uint32_t)A, b = id - o * (uint32_t)A;
                            if (w & 0x8000u) {                    // the state's row: n += 1
                                ++trace_states;
                                const uint32_t rid = ut_o * SL + lrow(o);
                                if (rsweep) atomicAdd(&CNTR[rid], 1u);
                                else if (atomicAdd(&CNTR[rid], 1u) == 0u) LIST[atomicAdd(&LISTN[0], 1u)] = (uint16_t)rid;
                            }
                            contrib_tr(qi(ut_o, o, b), p.lr * (td_o * ev), e_tr);
                            const double en = ev * p.gl;
                            if (in_lds) pc.TRE[pc.ixe_t(j, col)] = en;
                            else p.trace[pslot(p, j, lanev[u])] = en;
                        }
                    }
                }
            } else if constexpr (PAIRS) {
                if (train) pair_visit<A>(p, pc, lane, L.s, L.a, tcnt);
                pair_sweep(p, pc, lane, train ? tcnt : 0u, [&](uint32_t id, bool first, double ev) {
                    const uint32_t o = id / (uint32_t)A, b = id - o * (uint32_t)A;
                    if (first) {                              // the state's row: n += 1
                        ++trace_states;
                        const uint32_t rid = ut * SL + lrow(o);
                        if (rsweep) atomicAdd(&CNTR[rid], 1u);
                        else if (atomicAdd(&CNTR[rid], 1u) == 0u) LIST[atomicAdd(&LISTN[0], 1u)] = (uint16_t)rid;
                    }
                    contrib_tr(qi(ut, o, b), p.lr * (td * ev), e_tr);
                });
            } else {
                if (train) trace_visit<A>(p, lane, L.s, L.a, tcnt);
                const uint32_t nv = train ? tcnt : 0u;
                trace_states += nv;
                trace_sweep<A>(p, lane, nv,
                  [&](uint32_t o) {                            // once per visited state: its row count
                    const uint32_t rid = ut * SL + lrow(o);
                    if (rsweep) atomicAdd(&CNTR[rid], 1u);
                    else if (atomicAdd(&CNTR[rid], 1u) == 0u) LIST[atomicAdd(&LISTN[0], 1u)] = (uint16_t)rid;
                  },
                  [&](uint32_t o, uint32_t b, double ev) { contrib_tr(qi(ut, o, b), p.lr * (td * ev), e_tr); });
            }
            if constexpr (PAIRS) {
                // a non-finite td also moves the never-taken actions of every visited
                // state, whose E is 0: lr * (td * 0) is NaN (elegibility_traces_agent.rs:
                // 86-96 sweeps whole rows); the pair lists hold only taken actions
                if (POOL && train && !__builtin_isfinite(td)) {
                    // the lane's visited states are its pair bits: A == 4 bits per state
                    // (rare: kept rolled — unrolled it was 2.4k instructions inside the step loop)
                    const double dn = p.lr * (td * 0.0);
#pragma unroll 1
                    for (uint32_t wi = 0; wi < (uint32_t)PBW; ++wi) {
                        const uint32_t w = pbits_word(wi);
                        uint32_t m = w;
#pragma unroll 1
                        while (m) {
                            const uint32_t k = (uint32_t)__builtin_ctz(m) >> 2;
                            const uint32_t bits = (w >> (4u * k)) & 0xfu;
                            m &= ~(0xfu << (4u * k));
                            const uint32_t o = wi * 8u + k;
#pragma unroll 1
                            for (uint32_t b = 0; b < 4u; ++b)
                                if (!((bits >> b) & 1u)) contrib_tr(qi(ut, o, b), dn, e_tr);
                        }
                    }
                } else if (train && !__builtin_isfinite(td)) {
                    const double dn = p.lr * (td * 0.0);
                    auto id_at = [&](uint32_t j) -> uint32_t {
                        return j < pc.cap ? (uint32_t)pc.TRI[pc.ixi(j)] : (uint32_t)p.tlist[pslot(p, j, lane)];
                    };
                    for (uint32_t j = 0; j < tcnt; ++j) {
                        const uint32_t w = id_at(j);
                        if (!(w & 0x8000u)) continue;
                        const uint32_t o = (w & 0x7fffu) / (uint32_t)A;
                        uint32_t taken = 0;
                        if constexpr (PBITS) {
                            taken = (pbits_word((o * (uint32_t)A) >> 5) >> ((o * (uint32_t)A) & 31u)) & 0xfu;
                        } else {
                            for (uint32_t i = 0; i < tcnt; ++i) {
                                const uint32_t x = (id_at(i) & 0x7fffu) - o * (uint32_t)A;
                                if (x < (uint32_t)A) taken |= 1u << x;
                            }
                        }
                        for (uint32_t b = 0; b < (uint32_t)A; ++b)
                            if (!((taken >> b) & 1u)) contrib_tr(qi(ut, o, b), dn, e_tr);
                    }
                }
                if (train && term) {
                    if constexpr (!POOL) pair_clear(p, pc, lane, tcnt);
                    if constexpr (PBITS) {
#pragma unroll
                        for (int i = 0; i < PBW; ++i) pbits[i] = 0u;
                    }
                }
            }
            if (train && term) tcnt = 0;                  // the trace map is cleared
            __syncthreads();   // all contributions in, all Q reads done
            if (tid == 0) GCODE[0] = 0u;                  // read by every thread before the sweep
            if (rsweep) {
                for (uint32_t r = tid; r < (uint32_t)P * SL; r += nthr) settle_row(r, e_tr);
            } else {
                const uint32_t n_touched = LISTN[0];
                for (uint32_t i = tid; i < n_touched; i += nthr) settle_row(LIST[i], e_tr);
                __syncthreads();
                if (tid == 0) LISTN[0] = 0u;
            }
        }
        if constexpr (SPEC) {                     // fold the step's counter increments
            if (d_own != 0xffffffffu) {
                if (p.ucb_pack) {
                    const uint32_t w = NL[d_own];
                    NL[d_own] = ((w >> 16) + (w & 0xffffu)) << 16;
                } else {
                    NL[d_own] += (uint32_t)D16[d_own];
                    D16[d_own] = 0;
                }
            }
            if (tid == 0) { T[0] += T[1]; T[1] = 0ull; }
        }
        // Q_{t+1} complete before the next step's reads (one action per step: after
        // the next step's env step instead, below; reset-and-step reads Q first —
        // and a barrier between its deal and its reads measured 0.98x on cfg 5)
        if (!RLAMD_LATE_B3 || rs_on) __syncthreads();
        bool tr = false, ev = false;
        if constexpr (!INSTR && RLAMD_TAIL) {
            // one predicated block (no STEP / RESET branches): the STEP lanes'
            // bookkeeping computed for every lane, then every lane-state field written
            // once by a select — RESET lanes start an episode, idle lanes keep theirs
            if (train) {
                if (P == 2) L.dflag = !L.dflag;            // after_update
                if constexpr (!UCB) {                      // decay_epsilon: one select per lane
                    const double nw = L.eps * p.eps_dm - p.eps_ds;
                    L.eps = (term && !(p.eps_final > nw)) ? nw : L.eps;
                }
            }
            LaneRegs N = L;
            after_step<EPI>(p, N, s2, a2, r, term, tr, ev);   // term is false on RESET / idle lanes
            const bool act = doS || doR;
            L.epi_reward = doS ? N.epi_reward : (doR ? 0.0 : L.epi_reward);
            L.epi_len = doS ? N.epi_len : (doR ? 0u : L.epi_len);
            L.s = act ? s2 : L.s;
            L.a = act ? a2 : L.a;
            L.train_ep = doS ? N.train_ep : L.train_ep;
            L.mode = doS ? N.mode : L.mode;
            L.eval_left = doS ? N.eval_left : L.eval_left;
            L.need_reset = doS ? N.need_reset : (doR ? false : L.need_reset);
            tr = tr && doS;
            ev = ev && doS;
            if (tr) atomicAdd(RSUM, (unsigned long long)(FQ ? (int64_t)__builtin_rint(L.epi_reward * 65536.0)
                                                             : rint_i64_small(L.epi_reward * 65536.0)));
        } else if (doS) {
            if (train) {
                if (P == 2) L.dflag = !L.dflag;            // after_update
                if constexpr (!UCB) {                      // decay_epsilon: one select per lane
                    const double nw = L.eps * p.eps_dm - p.eps_ds;
                    L.eps = (term && !(p.eps_final > nw)) ? nw : L.eps;
                }
            }
            if (INSTR && p.rec) write_record(p, k, lane, fused ? 3u : 2u, L.s, L.a, s2, a2, r, term, td, mode_before);
            after_step<EPI>(p, L, s2, a2, r, term, tr, ev);
            // fixed point: the host also proved |episode reward| * 2^16 < 2^51
            // (delta_bound), so rint is the magic add
            if constexpr (RLAMD_RSUM_REG && !INSTR) {
                const int64_t rq = FQ ? (int64_t)__builtin_rint(L.epi_reward * 65536.0) : rint_i64_small(L.epi_reward * 65536.0);
                rsum_lane += tr ? rq : (int64_t)0;
            } else {
                if (tr) atomicAdd(RSUM, (unsigned long long)(FQ ? (int64_t)__builtin_rint(L.epi_reward * 65536.0)
                                                                 : rint_i64_small(L.epi_reward * 65536.0)));
            }
            if (INSTR && p.elog && (tr || ev)) log_episode(p, lane, L, tr);
        } else if (doR) {
            L.s = s2;
            L.a = a2;
            L.need_reset = false;
            L.epi_reward = 0.0;
            L.epi_len = 0;
            if (INSTR && p.rec) write_record(p, k, lane, 1u, s2, a2, 0u, 0u, 0.0, false, 0.0, mode_before);
        } else if (INSTR && p.rec && active) {
            write_record(p, k, lane, 0u, 0u, 0u, 0u, 0u, 0.0, false, 0.0, RL_MODE_DONE);
        }
        if constexpr (!RLAMD_EARLY_COUNT) {
            c_train += (uint32_t)__popcll(__ballot(train));
            c_tep += (uint32_t)__popcll(__ballot(tr));
            if (EPI > 0 || (EPI < 0 && p.episodic)) {   // run(): lanes only train, so no eval steps / episodes
                c_eval += (uint32_t)__popcll(__ballot(doS && !train));
                c_eep += (uint32_t)__popcll(__ballot(ev));
            }
        }
    }

    if (active) lane_store(p, lane, L);
    if constexpr (POOL) {
        const uint32_t nl = npool < lay.trc_cap ? npool : lay.trc_cap;
        for (uint32_t q = plid; q < nl; q += 64u) {
            uint32_t tg;
            double e;
            pool_get(q, tg, e);
            HT[q] = (uint16_t)tg;
            HE[q] = e;
        }
        if (plid == 0 && pwave) p.tcnt[plane0] = npool;
    } else {
        if constexpr (TRACES) { if (active) p.tcnt[lane] = tcnt; }
        if constexpr (PAIRS) { if (active) pair_cache_store(p, pc, lane, tcnt); }
    }
    {
        if constexpr (RLAMD_RSUM_REG && !INSTR) {
            const int64_t rw = wave_sum_i64(rsum_lane);
            if ((tid & 63u) == 0 && rw) atomicAdd(RSUM, (unsigned long long)rw);
        }
        const uint32_t c_done = (uint32_t)__popcll(__ballot(active && L.mode == RL_MODE_DONE));
        if ((tid & 63u) == 0) {
            if (c_train) atomicAdd(&ACC[0], (unsigned long long)c_train);
            if (c_eval) atomicAdd(&ACC[1], (unsigned long long)c_eval);
            if (c_tep) atomicAdd(&ACC[2], (unsigned long long)c_tep);
            if (c_eep) atomicAdd(&ACC[3], (unsigned long long)c_eep);
            if (c_done) atomicAdd(&ACC[5], (unsigned long long)c_done);
        }
        if constexpr (TRACES) {
            const int64_t ts = wave_sum_i64((int64_t)trace_states);
            if ((tid & 63u) == 0 && ts) atomicAdd(&ACC[7], (unsigned long long)ts);
        }
        flush_block(p, ACC);
    }

    // ---------------- emit this group's changes for the merge.  Fixed point:
    // ΔQ and group counts into replica blockIdx % n_rep of the SUM words ([PSA
    // sums][PSA group counts][SA dN][1 dt], folded by k_fold_replicas); f64: the
    // group's Q values into its slot (k_fq_merge_a / _b take the mean).
    int64_t *const dl = p.delta_rep + (uint64_t)(blockIdx.x % p.n_rep) * p.delta_words;
    __syncthreads();
    if constexpr (FQ) {
        uint64_t *const slot = p.qslot + (uint64_t)blockIdx.x * PSAL;
        for (uint32_t j = tid; j < PSAL; j += nthr) slot[j] = Q[j];
    } else {
        for (uint32_t j = tid; j < PSAL; j += nthr) {
            const uint32_t i = dense_of(j);
            const int64_t d = (int64_t)(Q[j] - (unsigned long long)p.q_base[i]);
            if (d) {
                atomicAdd((unsigned long long *)&dl[i], (unsigned long long)d);
                atomicAdd((unsigned long long *)&dl[PSA + i], 1ull);
            }
        }
    }
    if constexpr (UCB) {
        for (uint32_t i = tid; i < SA; i += nthr) {
            const int64_t d = SPEC ? (int64_t)(p.ucb_pack ? (NL[i] >> 16) : NL[i])
                                   : (int64_t)(N[lds_of(i)] - (unsigned long long)p.n_base[i]);
            if (d) atomicAdd((unsigned long long *)&dl[2 * PSA + i], (unsigned long long)d);
        }
        if (tid == 0) {
            const int64_t d = (int64_t)(T[0] - p.t_base[0]);
            if (d) atomicAdd((unsigned long long *)&dl[2 * PSA + SA], (unsigned long long)d);
        }
    }
}

template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, bool INSTR, bool FQ>
__global__ void __launch_bounds__(1024) k_train_shared(KParams p) {
    train_shared_body<ENV, AGENT, POLICY, SEL, ALGO, INSTR, FQ>(p);
}
// the throughput mode (rl_agent_run) with the episodic bookkeeping compiled out,
// as k_train_shared_o8<..., EPI = 0>
#ifndef RLAMD_SHARED_RUNMODE
#define RLAMD_SHARED_RUNMODE 1
#endif
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, bool FQ>
__global__ void __launch_bounds__(1024) k_train_shared_run(KParams p) {
    train_shared_body<ENV, AGENT, POLICY, SEL, ALGO, false, FQ, -1, -1, false, -1, 0>(p);
}
// Eligibility traces on the small tables (FrozenLake, CliffWalking: the pair
// bitmap) in groups of <= 256 lanes, at most 2 groups per CU (cfg 4: 2^17 lanes in
// 512 groups): 2 waves per SIMD is all the lanes give, so a wave may hold 256
// VGPRs — the sweep's interleaved rounds and the bitmap stay in registers instead
// of the 128-VGPR bound's scratch spills
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) k_train_shared_w(KParams p) {
    train_shared_body<ENV, AGENT, POLICY, SEL, ALGO, false, true>(p);
}
template <int ENV, int AGENT, int POLICY>
constexpr bool use_w() {
    return RLAMD_TRACES_W && AGENT == RL_AGENT_TRACES && POLICY != RL_POLICY_NEURAL &&
           (ENV == RL_ENV_CLIFF_WALKING || ENV == RL_ENV_FROZEN_LAKE || ENV == RL_ENV_FROZEN_LAKE_EDITED);
}
// the shared kernel for the agent's representation (nullptr: the fixed point
// cannot be proven for this variant, so the host never asks for it)
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, bool INSTR>
const void *shared_kernel(const KParams &p) {
    const bool run = RLAMD_SHARED_RUNMODE && !INSTR && !p.episodic;
    if (p.fq) return run ? (const void *)k_train_shared_run<ENV, AGENT, POLICY, SEL, ALGO, true>
                         : (const void *)k_train_shared<ENV, AGENT, POLICY, SEL, ALGO, INSTR, true>;
    if constexpr (fix_possible<AGENT, POLICY, SEL, ALGO>())
        return run ? (const void *)k_train_shared_run<ENV, AGENT, POLICY, SEL, ALGO, false>
                   : (const void *)k_train_shared<ENV, AGENT, POLICY, SEL, ALGO, INSTR, false>;
    return nullptr;
}
// Throughput variant at 8 waves per SIMD (<= 64 VGPRs, <= 96 SGPRs) for the
// learner groups whose LDS footprint allows 8 waves: one-step tabular
// FrozenLake / CliffWalking in the fixed point (proven range), and one-step
// eps-greedy Blackjack (single or double table) in the fixed point or in f64.
// The other variants would spill for no occupancy.
// MODE 1: fixed point; 2: fixed point with packed (sum, count) contributions; 3: f64
#ifndef RLAMD_O8_WAVES
#define RLAMD_O8_WAVES 8   // waves per SIMD the o8 kernels are compiled for
#endif
// EPI 0: the throughput mode (rl_agent_run, no episode target or eval interleave)
// with the episodic bookkeeping compiled out (fewer live scalars in the step loop);
// -1: either, by KParams::episodic (train / evaluate)
#ifndef RLAMD_O8_RUNMODE
#define RLAMD_O8_RUNMODE 1
#endif
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, int SLIP, int SWEEP, int MODE, int RS, int EPI>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(RLAMD_O8_WAVES, RLAMD_O8_WAVES))) k_train_shared_o8(KParams p) {
    train_shared_body<ENV, AGENT, POLICY, SEL, ALGO, false, MODE == 3, SLIP, SWEEP, MODE == 2, RS, EPI>(p);
}
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, int SLIP, int SWEEP, int MODE, int RS>
const void *o8_epi(const KParams &p) {
    if (RLAMD_O8_RUNMODE && !p.episodic)
        return (const void *)k_train_shared_o8<ENV, AGENT, POLICY, SEL, ALGO, SLIP, SWEEP, MODE, RS, 0>;
    return (const void *)k_train_shared_o8<ENV, AGENT, POLICY, SEL, ALGO, SLIP, SWEEP, MODE, RS, -1>;
}
// the reset-and-step schedule is compiled into the 8-wave kernels only where it
// is the measured better schedule (Blackjack, eps-greedy); elsewhere it runs on
// k_train_shared, and the 8-wave kernels carry no trace of it
template <int ENV, int SEL>
constexpr bool o8_has_reset_step() { return ENV == RL_ENV_BLACKJACK && SEL == RL_SEL_EPS_GREEDY; }
// the 8-wave kernel for (SLIP, SWEEP) and the agent's representation; nullptr: none
// (the caller takes k_train_shared)
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, int SLIP, int SWEEP, int RS>
const void *o8_kernel_rs(const KParams &p) {
    if (p.fq) {
        if constexpr (ENV == RL_ENV_BLACKJACK) return o8_epi<ENV, AGENT, POLICY, SEL, ALGO, SLIP, SWEEP, 3, RS>(p);
        return nullptr;
    }
    if constexpr (fix_possible<AGENT, POLICY, SEL, ALGO>())
        return p.pack_ok ? o8_epi<ENV, AGENT, POLICY, SEL, ALGO, SLIP, SWEEP, 2, RS>(p)
                         : o8_epi<ENV, AGENT, POLICY, SEL, ALGO, SLIP, SWEEP, 1, RS>(p);
    return nullptr;
}
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, int SLIP, int SWEEP>
const void *o8_kernel(const KParams &p) {
    if constexpr (o8_has_reset_step<ENV, SEL>()) {
        if (p.reset_step) return o8_kernel_rs<ENV, AGENT, POLICY, SEL, ALGO, SLIP, SWEEP, 1>(p);
    } else {
        if (p.reset_step && SEL == RL_SEL_EPS_GREEDY) return nullptr;
    }
    return o8_kernel_rs<ENV, AGENT, POLICY, SEL, ALGO, SLIP, SWEEP, 0>(p);
}
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO>
constexpr bool use_o8() {
    return ((ENV == RL_ENV_FROZEN_LAKE || ENV == RL_ENV_CLIFF_WALKING) && AGENT == RL_AGENT_ONE_STEP &&
            POLICY == RL_POLICY_TABULAR && !(SEL == RL_SEL_UCB && ALGO == RL_ALGO_EXPECTED_SARSA)) ||
           // Blackjack eps-greedy (compact rows: <= 35 KiB per group of 512, four groups
           // per CU): 67 VGPRs at the default bound left it at 3 groups per CU, i.e. a
           // second, one-third-full round of workgroups for cfg 5's 1024 groups per GPU
           (ENV == RL_ENV_BLACKJACK && AGENT == RL_AGENT_ONE_STEP && SEL == RL_SEL_EPS_GREEDY &&
            POLICY != RL_POLICY_NEURAL);
}

// ======================================================================== private
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, class NET = NetLane, bool PLAN = true>
__device__ __forceinline__ void run_private_lane(const KParams &p, const EnvTables &tabs, uint64_t lane,
                                                 LaneRegs &L, Counters &C, double *qb);

template <int ENV, int AGENT, int POLICY, int SEL, int ALGO>
__global__ void __launch_bounds__(256) k_train_private(KParams p) {
    using E = EnvDev<ENV>;
    constexpr int A = E::A;
    constexpr int P = POLICY == RL_POLICY_DOUBLE ? 2 : 1;
    constexpr bool UCB = SEL == RL_SEL_UCB;
    const uint32_t S = p.S, SA = S * (uint32_t)A;

    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const SmemLayout lay = smem_layout(ENV, P, UCB, AGENT == RL_AGENT_TRACES ? 1 : 0, S, A, p.n_start, 0u);
    uint32_t *TR = (uint32_t *)(smem + lay.tr);
    unsigned long long *ACC = (unsigned long long *)(smem + lay.st);
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    if (tid < STATS_W) ACC[tid] = 0ull;
    if constexpr (ENV != RL_ENV_TAXI && ENV != RL_ENV_BLACKJACK)
        for (uint32_t i = tid; i < SA; i += nthr) TR[i] = p.trans[i];
    __syncthreads();

    EnvTables tabs;
    tabs.trans = TR; tabs.cdf = p.start_cdf; tabs.n_start = p.n_start; tabs.max_steps = p.max_steps;
    tabs.th1 = p.th1; tabs.th2 = p.th2; tabs.th3 = p.th3; tabs.trunc_reward = p.trunc_reward;
    tabs.fixed_start = p.fixed_start;
    tabs.slippery = p.slippery;

    const uint64_t lane = (uint64_t)blockIdx.x * nthr + tid;
    const bool active = lane < p.L;
    LaneRegs L;
    Counters C;
    lane_load(p, lane, active, L);
    if (active)
        run_private_lane<ENV, AGENT, POLICY, SEL, ALGO>(p, tabs, lane, L, C,
                                                        p.q_priv ? p.q_priv + lane * (uint64_t)(P * SA) : nullptr);
    flush_stats(p, L, C, active, ACC);
}

// NeuralPolicy lanes with the bin's network (frozen_lake_neural.rs:130-134:
// DenseLayer(1, 32) -> leaky_relu6 -> DenseLayer(32, 4) -> linear on FrozenLake's
// scalar observation, one-step agents):
// each thread holds its lane's 196 f64 parameters in registers for the launch
// (one wave per SIMD: the 392 parameter registers and the step's temporaries fit
// the 512 of a lane at that occupancy), loaded once from the [param][lane] HBM
// layout and written back once.  k_train_private with NetLane reads the
// parameters three times per step and writes them once (6.3 KB per env-step,
// 421 GB per cfg 6 launch at 0.52 of HBM peak); here the step loop touches no
// parameter memory.  Same operations in the same order: bit-identical.
#ifndef RLAMD_NET_PAIR
#define RLAMD_NET_PAIR 1   // NeuralPolicy: the step's two predicts in one parameter pass
#endif
#ifndef RLAMD_NET_REGS
#define RLAMD_NET_REGS 1
#endif
template <int ENV, int AGENT, int SEL, int ALGO>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_train_private_net(KParams p) {
    using E = EnvDev<ENV>;
    constexpr int A = E::A;
    constexpr bool UCB = SEL == RL_SEL_UCB;
    const uint32_t S = p.S, SA = S * (uint32_t)A;

    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const SmemLayout lay = smem_layout(ENV, 1, UCB, 0, S, A, p.n_start, 0u);
    uint32_t *TR = (uint32_t *)(smem + lay.tr);
    unsigned long long *ACC = (unsigned long long *)(smem + lay.st);
    const uint32_t tid = threadIdx.x, nthr = blockDim.x;
    if (tid < STATS_W) ACC[tid] = 0ull;
    if constexpr (ENV != RL_ENV_TAXI && ENV != RL_ENV_BLACKJACK)
        for (uint32_t i = tid; i < SA; i += nthr) TR[i] = p.trans[i];
    __syncthreads();

    EnvTables tabs;
    tabs.trans = TR; tabs.cdf = p.start_cdf; tabs.n_start = p.n_start; tabs.max_steps = p.max_steps;
    tabs.th1 = p.th1; tabs.th2 = p.th2; tabs.th3 = p.th3; tabs.trunc_reward = p.trunc_reward;
    tabs.fixed_start = p.fixed_start;
    tabs.slippery = p.slippery;

    const uint64_t lane = (uint64_t)blockIdx.x * nthr + tid;
    const bool active = lane < p.L;
    LaneRegs L;
    Counters C;
    lane_load(p, lane, active, L);
    if (active)
        run_private_lane<ENV, AGENT, RL_POLICY_NEURAL, SEL, ALGO, NetBin<(uint32_t)A>, false>(p, tabs, lane, L, C,
                                                                                             nullptr);
    flush_stats(p, L, C, active, ACC);
}
// the register-resident network kernel exists for these instantiations; the host
// (and launch_train) also require the bin's shape and activations at run time
template <int ENV, int AGENT, int POLICY>
__host__ __device__ constexpr bool use_net_regs() {
    return RLAMD_NET_REGS && POLICY == RL_POLICY_NEURAL && AGENT == RL_AGENT_ONE_STEP && ENV == RL_ENV_FROZEN_LAKE;
}

// Private agents with small tables (KParams::priv_lpw != 0; FrozenLake 4x4 / 8x8,
// CliffWalking, single or double): the launch's lanes hold their Q tables in LDS.
// A block is 4 waves of priv_lpw lanes each (the other threads of a wave idle:
// cfg 7 19.9 ms per launch at 8 lanes per wave, 28.2 at 4, 31.4 at 16, 41.5 with Q
// in HBM — profiles/r05/private_lds_lpw_sweep.txt, cfg7_private_lds_ab.txt),
// its lanes' tables — one contiguous run of the lane-major q_priv — are copied in,
// the K steps read and write only LDS, and the tables go back at the end.  Each
// lane's slot is padded by two f64, so the slots of a wave's lanes start in
// different banks.  Private random gathers from HBM cost a 64-byte sector per
// 8-32 useful bytes (cfg 7: 7.5x the algorithmic traffic in the lane-major HBM form).
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO>
__global__ void __launch_bounds__(256) k_train_private_lds(KParams p) {
    using E = EnvDev<ENV>;
    constexpr int A = E::A;
    constexpr int P = POLICY == RL_POLICY_DOUBLE ? 2 : 1;
    constexpr bool UCB = SEL == RL_SEL_UCB;
    const uint32_t S = p.S, SA = S * (uint32_t)A, PSA = (uint32_t)P * SA, stride = PSA + 2u;

    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const SmemLayout lay = smem_layout(ENV, P, UCB, AGENT == RL_AGENT_TRACES ? 1 : 0, S, A, p.n_start, 0u);
    uint32_t *TR = (uint32_t *)(smem + lay.tr);
    unsigned long long *ACC = (unsigned long long *)(smem + lay.st);
    double *QS = (double *)(smem + align16(lay.total));
    const uint32_t tid = threadIdx.x, nthr = blockDim.x, lpw = p.priv_lpw, nl = (nthr >> 6) * lpw;
    const uint64_t lane0 = (uint64_t)blockIdx.x * nl;
    const uint32_t nv = lane0 + nl <= p.L ? nl : (uint32_t)(p.L - lane0);   // lanes of this block
    if (tid < STATS_W) ACC[tid] = 0ull;
    if constexpr (ENV != RL_ENV_TAXI && ENV != RL_ENV_BLACKJACK)
        for (uint32_t i = tid; i < SA; i += nthr) TR[i] = p.trans[i];
    const double *qg = p.q_priv + lane0 * PSA;                   // the block's tables, contiguous
    for (uint32_t l = 0; l < nv; ++l)
        for (uint32_t e = tid; e < PSA; e += nthr) QS[l * stride + e] = qg[(uint64_t)l * PSA + e];
    __syncthreads();

    EnvTables tabs;
    tabs.trans = TR; tabs.cdf = p.start_cdf; tabs.n_start = p.n_start; tabs.max_steps = p.max_steps;
    tabs.th1 = p.th1; tabs.th2 = p.th2; tabs.th3 = p.th3; tabs.trunc_reward = p.trunc_reward;
    tabs.fixed_start = p.fixed_start;
    tabs.slippery = p.slippery;

    const uint32_t slot = (tid >> 6) * lpw + (tid & 63u);
    const uint64_t lane = lane0 + slot;
    const bool active = (tid & 63u) < lpw && slot < nv;
    LaneRegs L;
    Counters C;
    lane_load(p, lane, active, L);
    if (active) run_private_lane<ENV, AGENT, POLICY, SEL, ALGO>(p, tabs, lane, L, C, QS + slot * stride);
    __syncthreads();
    double *qo = p.q_priv + lane0 * PSA;
    for (uint32_t l = 0; l < nv; ++l)
        for (uint32_t e = tid; e < PSA; e += nthr) qo[(uint64_t)l * PSA + e] = QS[l * stride + e];
    flush_stats(p, L, C, active, ACC);
}

// One private lane as a reference agent: Policy + ActionSelection + the TD update,
// over the lane's f64 Q / UCB counters / trace set / network in HBM.  Used by the
// private training kernel (K steps per launch) and by the per-call Agent surface
// (k_agent_call: rl_agent_get_action / rl_agent_update).
// PLAN: the Dyna model code compiled in (k_train_private_net, whose registers hold
// the network, runs only agents without planning: launch_train)
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, class NET = NetLane, bool PLAN = true>
struct PrivAgent {
    using E = EnvDev<ENV>;
    static constexpr int A = E::A;
    static constexpr int P = POLICY == RL_POLICY_DOUBLE ? 2 : 1;
    static constexpr bool UCB = SEL == RL_SEL_UCB;
    static constexpr bool NEURAL = POLICY == RL_POLICY_NEURAL;
    const KParams &p;
    const uint64_t lane, Ls;
    const uint32_t SA;
    LaneRegs &L;
    Counters &C;
    uint64_t t;        // UCB t (upper_confidence_bound.rs:13)
    uint32_t tcnt;     // traces: visited states this episode
    NET net;           // the network's parameters (NeuralPolicy): HBM (NetLane) or registers (NetRegs)
    NetCache<A> nc;
    NetCache<A> nc_b;  // the second entry of a paired predict (prefetch_pair)
    double *const qb;
    // Dyna (InternalModelAgent): the model's entry count for the launch, and the
    // slot word of the step's (s, a) read ahead of the step (model_prefetch)
    uint32_t mc = 0, jpf = 0;
    bool jpf_ok = false;   // the lane's Q block [P][S][A]: in HBM (q_priv, lane-major) or its LDS slot

    __device__ __forceinline__ PrivAgent(const KParams &p_, uint64_t lane_, LaneRegs &L_, Counters &C_, double *qb_)
        : p(p_), lane(lane_), Ls(p_.L), SA(p_.S * (uint32_t)A), L(L_), C(C_),
          t(UCB ? p_.t_priv[lane_] : 0), tcnt(AGENT == RL_AGENT_TRACES ? p_.tcnt[lane_] : 0u),
          net(NET::template make<A>(p_, lane_)), qb(qb_) {
        if (PLAN && p.plan_steps) mc = p.mcnt[lane];
    }
    __device__ __forceinline__ void store() {
        if (UCB) p.t_priv[lane] = t;
        if (AGENT == RL_AGENT_TRACES) p.tcnt[lane] = tcnt;
        if constexpr (NEURAL) net.store(p, lane);
        if (PLAN && p.plan_steps) p.mcnt[lane] = mc;
    }
    // the model slot of (s, a), read at the start of a training step so its HBM
    // round trip overlaps the env step, the selection and the update
    __device__ __forceinline__ void model_prefetch(uint32_t s, uint32_t a) {
        jpf = p.mslot[lane * (uint64_t)SA + s * A + a];
        jpf_ok = true;
    }
    // lane-major tables (rl_kparams.h): the lane's Q block [P][S][A], its UCB counts [S][A]
    __device__ __forceinline__ double &qref(uint32_t idx) const { return qb[idx]; }
    __device__ __forceinline__ uint64_t &nref(uint32_t idx) const { return p.n_priv[lane * (uint64_t)SA + idx]; }
    // row s of table tbl: A consecutive f64, 16-byte aligned (P*S*A and A even for every env)
    __device__ __forceinline__ void row(uint32_t tbl, uint32_t s, double (&v)[A]) const {
        if constexpr (A % 2 == 0) {
            const double2 *r = (const double2 *)__builtin_assume_aligned(&qref(tbl * SA + s * A), 16);
#pragma unroll
            for (int i = 0; i < A / 2; ++i) {
                const double2 x = r[i];
                v[2 * i] = x.x;
                v[2 * i + 1] = x.y;
            }
        } else {
#pragma unroll
            for (int i = 0; i < A; ++i) v[i] = qref(tbl * SA + s * A + i);
        }
    }
    // Policy::predict (tabular_policy.rs:27-29, double_tabular_policy.rs:31-40, neural_policy.rs:43-47)
    __device__ __forceinline__ void predict(uint32_t s, double (&v)[A]) {
        if constexpr (NEURAL) {
            if constexpr (RLAMD_NET_PAIR) nc.take(nc_b, s);
            nc.get(p, net, s);
#pragma unroll
            for (int i = 0; i < A; ++i) v[i] = nc.y[i];
            return;
        }
        row(0u, s, v);
        if constexpr (P == 2) {
            double w[A];
            row(1u, s, w);
#pragma unroll
            for (int i = 0; i < A; ++i) v[i] = (v[i] + w[i]) / 2.0;
        }
    }
    // Policy::get_values of table `tbl` (double policy: flag ? alpha : beta)
    __device__ __forceinline__ void values(uint32_t tbl, uint32_t s, double (&v)[A]) {
        if constexpr (NEURAL) {
            predict(s, v);
        } else {
            row(tbl, s, v);
        }
    }
    // Policy::update with x = td (one-step) or td * E[o][b] (traces)
    __device__ __forceinline__ void pol_update(uint32_t tbl, uint32_t s, uint32_t a, double x) {
        if constexpr (NEURAL) {
            if constexpr (RLAMD_NET_PAIR) nc.take(nc_b, s);
            net_policy_update<A>(p, net, nc, s, a, x);
            nc_b.invalidate();                                  // the parameters changed
        } else {
            double &q = qref(tbl * SA + s * A + a);             // tabular_policy.rs:36
            q = q + p.lr * x;
        }
    }
    // NeuralPolicy training step: the step's two predicts — get_action(s2) and
    // update's get_values(s) — in one pass over the parameters (the same values:
    // nothing changes the parameters between them)
    __device__ __forceinline__ void prefetch_pair(uint32_t s2, uint32_t s) {
        if constexpr (NEURAL && RLAMD_NET_PAIR) nc.get_pair(p, net, s2, nc_b, s);
    }
    // Agent::get_action (one_step_agent.rs:48-51) with the reference's immediate UCB increments
    __device__ __forceinline__ uint32_t select(uint32_t s) {
        double v[A];
        predict(s, v);
        if constexpr (!UCB) {
            if (L.eps != 0.0 && eps_test(L.rng, L.eps)) return uniform_action<A>(L.rng);
            return argmax<A>(v);
        } else {
            const double lnt = rl_log((double)t);
            double u[A];
#pragma unroll
            for (int i = 0; i < A; ++i)
                u[i] = ucb_value(v[i], p.ucb_c, lnt, (double)nref(s * A + i));
            const uint32_t a = argmax<A>(u);
            nref(s * A + a) += 1ull;
            t += 1;
            return a;
        }
    }
    // Agent::update (one_step_agent.rs:53-86 / elegibility_traces_agent.rs:61-104)
    // against the lane's current Q, with after_update and the termination hooks
    __device__ __forceinline__ double update(uint32_t s, uint32_t a, double r, bool term, uint32_t s2, uint32_t a2) {
        const uint32_t vt = (P == 2 && !L.dflag) ? 1u : 0u;
        const uint32_t ut = (P == 2 && L.dflag) ? 1u : 0u;
        double q2[A], pr[A];
        values(vt, s2, q2);
#pragma unroll
        for (int i = 0; i < A; ++i) pr[i] = 0.0;
        if constexpr (ALGO == RL_ALGO_EXPECTED_SARSA) {
            if constexpr (!UCB) {
                eps_probs<A>(L.eps, q2, pr);
            } else {
                const double lnt = rl_log((double)t);
                double sum = 0.0;
#pragma unroll
                for (int i = 0; i < A; ++i) {
                    pr[i] = ucb_value(q2[i], p.ucb_c, lnt, (double)nref(s2 * A + i));
                    sum += pr[i];
                }
#pragma unroll
                for (int i = 0; i < A; ++i) pr[i] /= sum;
            }
        }
        const double fq = future_q<ALGO, A>(q2, a2, pr);
        double qa;
        if constexpr (NEURAL) {
            double qs[A];
            values(vt, s, qs);
            qa = pick<A>(qs, a);
        } else {
            qa = qref(vt * SA + s * A + a);
        }
        const double td = r + p.gamma * fq - qa;
        if constexpr (AGENT == RL_AGENT_ONE_STEP) {
            pol_update(ut, s, a, td);
        } else {
            // the sweep runs in first-visit (slot) order: order-free for the
            // tabular policies, and the oracle's order for the neural one
            trace_visit<A>(p, lane, s, a, tcnt);
            C.trace_states += tcnt;
            trace_sweep<A>(p, lane, tcnt, [](uint32_t) {},
                           [&](uint32_t o, uint32_t b, double ev) { pol_update(ut, o, b, td * ev); });
            if (term) tcnt = 0;
        }
        if (P == 2) L.dflag = !L.dflag;                        // after_update
        if constexpr (!UCB) { if (term) L.eps = decay_eps(p, L.eps); }
        return td;
    }
    // the training update as the agent's own update() does it: the inner agent's,
    // then for InternalModelAgent (src/agent/internal_model_agent.rs:47-77)
    // model.add_info, which keeps the first (s', r) seen for (s, a)
    // (random_model.rs:34-38), and planning_steps replays of a uniformly drawn
    // entry (gen_range, :29-31) through get_action + update(terminated = false)
    __device__ __forceinline__ double train_update(uint32_t s, uint32_t a, double r, bool term, uint32_t s2,
                                                   uint32_t a2) {
        const double td = update(s, a, r, term, s2, a2);
        if (PLAN && p.plan_steps) {
            const uint32_t key = s * A + a;
            uint4 *const mrec = p.mrec + lane * (uint64_t)SA;     // the lane's model, lane-major
            uint32_t *const mslot = p.mslot + lane * (uint64_t)SA;
            // mslot[key] = the entry's index + 1, 0 = not in the model (the host clears
            // the words when it empties the model)
            const uint32_t j0 = jpf_ok ? jpf : mslot[key];
            jpf_ok = false;
            if (j0 == 0u) {
                const uint64_t rb = (uint64_t)__double_as_longlong(r);
                mrec[mc] = make_uint4(key, s2, (uint32_t)rb, (uint32_t)(rb >> 32));
                mslot[key] = mc + 1u;
                ++mc;
            }
            if constexpr (!UCB && !NEURAL && RLAMD_PLAN_PF) {
                // eps-greedy draws depend on the stream and eps only, never on Q: a batch
                // of planning steps takes its draws first (gen_index, the eps test, the
                // exploring action: the order of the loop below), issues its model reads
                // together, then runs the selections and updates in order — the exploit
                // argmax reads Q after the previous planning updates, as the loop does
                // RLAMD_PLAN_PB steps per batch (cfg 7, 10 planning steps: 4 -> 20.28 ms per
                // launch, 8 -> 19.70, 16 -> 18.99, profiles/r05/cfg7_plan_batch.txt)
                constexpr uint32_t PB = RLAMD_PLAN_PB;
                for (uint32_t i0 = 0; i0 < p.plan_steps; i0 += PB) {
                    const uint32_t nb = p.plan_steps - i0 < PB ? p.plan_steps - i0 : PB;
                    uint4 m[PB];
                    std::conditional_t<(PB > 8), uint64_t, uint32_t> acts = 0;                        // 4 bits per step: action + 1, 0 = exploit
#pragma unroll
                    for (uint32_t b = 0; b < PB; ++b) {
                        if (b < nb) {
                            const uint32_t j = gen_index(L.rng, mc);
                            uint32_t a1 = 0;
                            if (L.eps != 0.0 && eps_test(L.rng, L.eps)) a1 = uniform_action<A>(L.rng) + 1u;
                            acts |= (decltype(acts))a1 << (4u * b);
                            m[b] = mrec[j];                    // one 16-byte read each, all in flight
                        }
                    }
#pragma unroll
                    for (uint32_t b = 0; b < PB; ++b) {
                        if (b < nb) {
                            const uint32_t pk = m[b].x, ps2 = m[b].y;
                            const double pr = __longlong_as_double((long long)(((uint64_t)m[b].w << 32) | m[b].z));
                            const uint32_t a1 = (uint32_t)(acts >> (4u * b)) & 0xfu;
                            uint32_t na;
                            if (a1) {
                                na = a1 - 1u;
                            } else {
                                double v[A];
                                predict(ps2, v);
                                na = argmax<A>(v);
                            }
                            update(pk / (uint32_t)A, pk % (uint32_t)A, pr, false, ps2, na);
                        }
                    }
                }
            } else {
                for (uint32_t i = 0; i < p.plan_steps; ++i) {
                    const uint32_t j = gen_index(L.rng, mc);
                    const uint4 m = mrec[j];                         // one 16-byte read
                    const uint32_t pk = m.x;
                    const uint32_t ps2 = m.y;
                    const double pr = __longlong_as_double((long long)(((uint64_t)m.w << 32) | m.z));
                    const uint32_t na = select(ps2);
                    update(pk / (uint32_t)A, pk % (uint32_t)A, pr, false, ps2, na);
                }
            }
        }
        return td;
    }
};

// one private lane (a whole reference agent) for K synchronous steps, its Q at qb
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, class NET, bool PLAN>
__device__ __forceinline__ void run_private_lane(const KParams &p, const EnvTables &tabs, uint64_t lane,
                                                 LaneRegs &L, Counters &C, double *qb) {
    using E = EnvDev<ENV>;
    PrivAgent<ENV, AGENT, POLICY, SEL, ALGO, NET, PLAN> ag(p, lane, L, C, qb);
    for (uint32_t k = 0; k < p.K; ++k) {
        if (L.mode == RL_MODE_DONE) {
            if (p.rec) write_record(p, k, lane, 0u, 0u, 0u, 0u, 0u, 0.0, false, 0.0, RL_MODE_DONE);
            continue;
        }
        if (L.need_reset) {                       // RESET step: src/agent.rs:83-84
            L.s = E::reset(L.z, L.rng, tabs);
            L.ready = true;
            L.a = ag.select(L.s);
            L.need_reset = false;
            L.epi_reward = 0.0;
            L.epi_len = 0;
            if (p.rec) write_record(p, k, lane, 1u, L.s, L.a, 0u, 0u, 0.0, false, 0.0, L.mode);
            continue;
        }
        const uint32_t mode_before = L.mode;      // STEP: src/agent.rs:88-101
        if (PLAN && p.plan_steps && L.mode == RL_MODE_TRAIN) ag.model_prefetch(L.s, L.a);
        uint32_t s2 = 0;
        double r = 0.0;
        bool term = false;
        {
            uint32_t pos = L.s;
            E::step(pos, L.z, L.a, L.rng, tabs, s2, r, term);
            if (term) L.ready = false;
        }
        if constexpr (POLICY == RL_POLICY_NEURAL && AGENT == RL_AGENT_ONE_STEP)
            if (L.mode == RL_MODE_TRAIN) ag.prefetch_pair(s2, L.s);
        const uint32_t a2 = ag.select(s2);
        double td = 0.0;
        if (L.mode == RL_MODE_TRAIN) {
            td = ag.train_update(L.s, L.a, r, term, s2, a2);
            C.n_train++;
        } else {
            C.n_eval++;
        }
        if (p.rec) write_record(p, k, lane, 2u, L.s, L.a, s2, a2, r, term, td, mode_before);
        bool tr, ev;
        after_step(p, L, s2, a2, r, term, tr, ev);
        if (p.elog && (tr || ev)) log_episode(p, lane, L, tr);
        C.n_tep += tr ? 1u : 0u;
        C.n_eep += ev ? 1u : 0u;
        C.rsum += tr ? (int64_t)__builtin_rint(L.epi_reward * 65536.0) : (int64_t)0;
    }
    lane_store(p, lane, L);
    ag.store();
}

// The per-call Agent surface (trait Agent, src/agent.rs:52-62) on private lanes
// [call_lane0, call_lane0 + call_n): CALL_GET_ACTION runs get_action(s) (the
// selector's draws come from the lane's stream, which the lane's Env view shares:
// one stream per lane, as thread_rng is one per thread), CALL_UPDATE runs
// update(s, a, r, term, s2, a2) and returns the TD error.  One thread per lane;
// the lane's record is read and written back around the call.
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO>
__global__ void __launch_bounds__(256) k_agent_call(KParams p) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.call_n) return;
    const uint64_t lane = (uint64_t)p.call_lane0 + i;
    if (lane >= p.L) return;
    LaneRegs L;
    Counters C;
    lane_load(p, lane, true, L);
    constexpr int P = POLICY == RL_POLICY_DOUBLE ? 2 : 1;
    PrivAgent<ENV, AGENT, POLICY, SEL, ALGO> ag(p, lane, L, C,
                                               p.q_priv ? p.q_priv + lane * (uint64_t)(P * p.S * EnvDev<ENV>::A) : nullptr);
    const AgentCall &c = p.call;
    if (p.call_op == CALL_GET_ACTION) {
        c.action_out[i] = ag.select(c.s[i]);
    } else {
        c.td_out[i] = ag.train_update(c.s[i], c.a[i], c.r[i], c.term[i] != 0, c.s2[i], c.a2[i]);
    }
    lane_store(p, lane, L);
    ag.store();
}

// ---------------------------------------------------------------- launch table
template <int ENV, int AGENT, int POLICY, int SEL, int ALGO, int PRIV>
hipError_t launch_train(const KParams &p, dim3 grid, dim3 block, size_t smem, hipStream_t stream, int *occ) {
    const bool instr = p.rec != nullptr || p.elog != nullptr;
    const void *k = nullptr;
    if constexpr (PRIV) {
        if (p.call_op != CALL_NONE) {   // per-call Agent surface: one thread per lane, no LDS
            if (occ) { *occ = 0; return hipSuccess; }
            void *args[] = {(void *)&p};
            return hipLaunchKernel((const void *)k_agent_call<ENV, AGENT, POLICY, SEL, ALGO>,
                                   dim3((p.call_n + 255) / 256), dim3(256), args, 0, stream);
        }
        k = (const void *)k_train_private<ENV, AGENT, POLICY, SEL, ALGO>;
        if constexpr (POLICY != RL_POLICY_NEURAL && ENV != RL_ENV_TAXI && ENV != RL_ENV_BLACKJACK)
            if (p.priv_lpw) k = (const void *)k_train_private_lds<ENV, AGENT, POLICY, SEL, ALGO>;
        if constexpr (use_net_regs<ENV, AGENT, POLICY>())
            if (p.net_regs && p.plan_steps == 0) k = (const void *)k_train_private_net<ENV, AGENT, SEL, ALGO>;
    } else if (instr) {
        k = shared_kernel<ENV, AGENT, POLICY, SEL, ALGO, true>(p);
    } else {
        if constexpr (use_o8<ENV, AGENT, POLICY, SEL, ALGO>()) {
            // the map's slippery flag (FrozenLake) and the settle form (every entry
            // owned by one thread when P*S*A <= block size) as compile-time constants
            const bool sw = p.P * p.S * p.A <= block.x;
            if constexpr (ENV == RL_ENV_FROZEN_LAKE) {
                if (!p.slippery) k = sw ? o8_kernel<ENV, AGENT, POLICY, SEL, ALGO, 0, 1>(p)
                                        : o8_kernel<ENV, AGENT, POLICY, SEL, ALGO, 0, -1>(p);
                else k = sw ? o8_kernel<ENV, AGENT, POLICY, SEL, ALGO, 1, 1>(p)
                            : o8_kernel<ENV, AGENT, POLICY, SEL, ALGO, 1, -1>(p);
            } else {
                k = sw ? o8_kernel<ENV, AGENT, POLICY, SEL, ALGO, -1, 1>(p)
                       : o8_kernel<ENV, AGENT, POLICY, SEL, ALGO, -1, -1>(p);
            }
        } else if constexpr (use_w<ENV, AGENT, POLICY>()) {
            // 256 CUs: <= 512 groups keeps the grid at <= 2 groups (2 waves per SIMD) per CU
            if (p.fq && block.x <= 256 && grid.x <= 512) k = (const void *)k_train_shared_w<ENV, AGENT, POLICY, SEL, ALGO>;
        }
        if (!k) k = shared_kernel<ENV, AGENT, POLICY, SEL, ALGO, false>(p);
    }
    if (!k) return hipErrorInvalidValue;   // the fixed point for a variant it cannot prove
    if (smem > 64 * 1024) {   // gfx950: a workgroup may use up to the CU's 160 KiB of LDS
        const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
        if (e != hipSuccess) return e;
    }
    if (occ) return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, k, (int)(block.x * block.y * block.z), smem);
    void *args[] = {(void *)&p};
    return hipLaunchKernel(k, grid, block, args, smem, stream);
}

// RLAMD_ONLY=ag,po,se,al,pr (experiment builds, scripts/build_variant.sh): only this
// (agent, policy, selector, algorithm, private) instantiation, so a timing variant
// of one kernel compiles in a minute instead of the whole table's ten
#ifdef RLAMD_ONLY
constexpr int kOnly[5] = {RLAMD_ONLY};
constexpr bool only_ok(int ag, int po, int se, int al, int pr) {
    return ag == kOnly[0] && po == kOnly[1] && se == kOnly[2] && al == kOnly[3] && pr == kOnly[4];
}
#else
constexpr bool only_ok(int, int, int, int, int) { return true; }
#endif
template <int ENV>
train_launch_fn train_table_entry(int agent, int policy, int sel, int algo, int priv) {
#define RLAMD_E(AG, PO, SE, AL, PR)                                                                \
    if constexpr (only_ok(AG, PO, SE, AL, PR))                                                     \
        if (agent == AG && policy == PO && sel == SE && algo == AL && priv == PR)                  \
            return &launch_train<ENV, AG, PO, SE, AL, PR>;
#define RLAMD_E1(AG, PO, SE, AL) RLAMD_E(AG, PO, SE, AL, 0) RLAMD_E(AG, PO, SE, AL, 1)
#define RLAMD_E2(AG, PO, SE)                                                                       \
    RLAMD_E1(AG, PO, SE, RL_ALGO_SARSA) RLAMD_E1(AG, PO, SE, RL_ALGO_QLEARNING)                     \
    RLAMD_E1(AG, PO, SE, RL_ALGO_EXPECTED_SARSA)
#define RLAMD_E3(AG, PO) RLAMD_E2(AG, PO, RL_SEL_EPS_GREEDY) RLAMD_E2(AG, PO, RL_SEL_UCB)
#define RLAMD_E4(AG) RLAMD_E3(AG, RL_POLICY_TABULAR) RLAMD_E3(AG, RL_POLICY_DOUBLE)
    RLAMD_E4(RL_AGENT_ONE_STEP)
    RLAMD_E4(RL_AGENT_TRACES)
    // NeuralPolicy: private agents only
#define RLAMD_N2(AG, SE)                                                                           \
    RLAMD_E(AG, RL_POLICY_NEURAL, SE, RL_ALGO_SARSA, 1) RLAMD_E(AG, RL_POLICY_NEURAL, SE, RL_ALGO_QLEARNING, 1) \
    RLAMD_E(AG, RL_POLICY_NEURAL, SE, RL_ALGO_EXPECTED_SARSA, 1)
    RLAMD_N2(RL_AGENT_ONE_STEP, RL_SEL_EPS_GREEDY) RLAMD_N2(RL_AGENT_ONE_STEP, RL_SEL_UCB)
    RLAMD_N2(RL_AGENT_TRACES, RL_SEL_EPS_GREEDY) RLAMD_N2(RL_AGENT_TRACES, RL_SEL_UCB)
#undef RLAMD_N2
#undef RLAMD_E4
#undef RLAMD_E3
#undef RLAMD_E2
#undef RLAMD_E1
#undef RLAMD_E
    return nullptr;
}

}  // namespace rlamd

// rl_host.cpp — host runtime behind include/rl.h: env table construction,
// device memory layout, launch sequencing, the group merge, recording,
// timing.  Everything compute-bearing runs in the gfx950 kernels; this file
// only allocates, copies and launches.  There is no CPU fallback: without a
// HIP device every compute entry point returns RL_E_HIP.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "rl_kparams.h"
#include "rl_taxi.h"

using namespace rlamd;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPC(expr)                                                                                 \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(e_ == hipErrorOutOfMemory ? RL_E_OOM : RL_E_HIP,                           \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                        \
    } while (0)

// ------------------------------------------------------------------ env tables
// The product's own construction of the reference envs (an independent
// restatement from the oracle's and from tests/golden/make_tables.py).
struct EnvHost {
    int kind = 0;
    uint32_t S = 0, A = 0, max_steps = 0;
    std::vector<uint32_t> trans;  // packed, see rl_device.h EnvDev<>
    std::vector<double> start;    // initial-state distribution
    std::vector<double> cdf;      // running sum of `start` (categorical_sample, utils.rs:33-43)
    double th1 = 0, th2 = 0, th3 = 0, trunc_reward = 0;
    int32_t fixed_start = -1;     // categorical_sample over `cdf` is constant (single start state)
    int32_t slippery = 0;         // FrozenLake with stochastic rows
    const char *const *map = nullptr;   // FrozenLake / FrozenLakeEdited grid (n x n)
    int n = 0;
};

const char *const kFL4[] = {"SFFF", "FHFH", "FFFH", "HFFG"};                     // frozen_lake.rs:23
const char *const kFL8[] = {"SFFFFFFF", "FFFFFFFF", "FFFHFFFF", "FFFFFHFF",       // frozen_lake.rs:25-28
                            "FFFHFFFF", "FHHFFFHF", "FHFFHFHF", "FFFHFFFG"};
const char *const kTaxiMap[] = {"+---------+", "|R: | : :G|", "| : | : : |", "| : : : : |",
                                "| | : | : |", "|Y| : |B: |", "+---------+"};   // taxi.rs:22-30
const int kTaxiLocs[4][2] = {{0, 0}, {0, 4}, {4, 0}, {4, 3}};                   // taxi.rs:31

// utils::inc (src/utils.rs:53-76): 0 LEFT, 1 DOWN, 2 RIGHT, 3 UP, clamped
void grid_move(int nrow, int ncol, int row, int col, int a, int &nr, int &nc) {
    nr = row;
    nc = col;
    switch (a) {
    case 0: nc = std::max(col - 1, 0); break;
    case 1: nr = std::min(row + 1, nrow - 1); break;
    case 2: nc = std::min(col + 1, ncol - 1); break;
    case 3: nr = std::max(row - 1, 0); break;
    default: break;
    }
}

// FrozenLakeTerrain of a cell / of the neighbour in direction a, WALL off the
// grid (src/env/frozen_lake_edited.rs get_obs :115-144, get_terrain :146-162)
enum { kStart = 0, kWall = 1, kHole = 2, kGround = 3, kGoal = 4 };
int terrain(const char *const *map, int row, int col) {
    const char ch = map[row][col];
    return ch == 'S' ? kStart : ch == 'G' ? kGoal : ch == 'H' ? kHole : kGround;
}
int neighbour(const char *const *map, int n, int row, int col, int a) {
    switch (a) {
    case 0: return col == 0 ? kWall : terrain(map, row, col - 1);
    case 1: return row == n - 1 ? kWall : terrain(map, row + 1, col);
    case 2: return col == n - 1 ? kWall : terrain(map, row, col + 1);
    default: return row == 0 ? kWall : terrain(map, row - 1, col);
    }
}
double terrain_value(int t) {   // FrozenLakeTerrain::value (frozen_lake_edited.rs:18-28)
    return t == kHole ? -1.0 : t == kWall ? -0.5 : t == kStart ? 0.0 : t == kGround ? 0.5 : 1.0;
}

void finish_cdf(EnvHost &e) {
    e.cdf.resize(e.start.size());
    double b = 0.0;
    for (size_t i = 0; i < e.start.size(); ++i) {
        b += e.start[i];
        e.cdf[i] = b;
    }
    // first i with cdf[i] > u for every u in [0, 1 - 2^-52]: fixed when all
    // earlier sums are 0 and cdf[i] exceeds the largest uniform
    e.fixed_start = -1;
    for (size_t i = 0; i < e.cdf.size(); ++i) {
        if (e.cdf[i] == 0.0) continue;
        if (e.cdf[i] > 1.0 - 0x1p-52) e.fixed_start = (int32_t)i;
        break;
    }
}

// categorical_sample over the cdf (utils.rs:33-43): first i with cdf[i] > u, else 0
uint32_t linear_sample(const std::vector<double> &cdf, double u) {
    for (size_t i = 0; i < cdf.size(); ++i)
        if (cdf[i] > u) return (uint32_t)i;
    return 0;
}
// rl_taxi.h taxi_start (three probes) equals the linear search at every
// boundary: each c_k and its neighbours, and the u around each k/300 where the
// first probe moves (between boundaries both are constant).  Checked once.
bool taxi_start_checked(const EnvHost &e) {
    static int ok = -1;
    if (ok >= 0) return ok == 1;
    std::vector<double> us = {0.0, std::nextafter(1.0, 0.0)};
    auto around = [&](double x) {
        double lo = x, hi = x;
        for (int i = 0; i < 8; ++i) { lo = std::nextafter(lo, 0.0); hi = std::nextafter(hi, 1.0); us.push_back(lo); us.push_back(hi); }
        us.push_back(x);
    };
    for (double c : e.cdf) if (c > 0.0 && c < 1.0) around(c);
    for (int j = 1; j < 300; ++j) around((double)j / 300.0);
    ok = 1;
    for (double u : us)
        if (u >= 0.0 && u < 1.0 && taxi_start(e.cdf.data(), u) != linear_sample(e.cdf, u)) ok = 0;
    return ok == 1;
}

int build_env(const rl_env_config &c, EnvHost &e) {
    e = EnvHost();
    e.kind = c.kind;
    e.max_steps = c.max_steps;
    if (c.kind == RL_ENV_FROZEN_LAKE || c.kind == RL_ENV_FROZEN_LAKE_EDITED) {
        const char *const *map = c.map8x8 ? kFL8 : kFL4;
        const int n = c.map8x8 ? 8 : 4;
        const bool edited = c.kind == RL_ENV_FROZEN_LAKE_EDITED;
        e.map = map;
        e.n = n;
        e.S = n * n;
        e.A = 4;
        e.trans.assign(e.S * 4, 0);
        int n_start = 0;
        for (int i = 0; i < n * n; ++i) n_start += map[i / n][i % n] == 'S';
        e.start.assign(e.S, 0.0);
        for (int i = 0; i < n * n; ++i)
            if (map[i / n][i % n] == 'S') e.start[i] = 1.0 / n_start;
        auto outcome = [&](int row, int col, int a) -> uint32_t {
            int nr, nc;
            grid_move(n, n, row, col, a, nr, nc);
            if (edited) {   // update_probability_matrix (frozen_lake_edited.rs:94-113): judged by
                            // the terrain in the moved direction; 10.0 onto G, else -1.0
                const int t = neighbour(map, n, row, col, a);
                return (uint32_t)(nr * n + nc) | (t == kGoal ? 64u : 0u) | ((t == kGoal || t == kHole) ? 128u : 0u);
            }
            const char ch = map[nr][nc];
            return (uint32_t)(nr * n + nc) | (ch == 'G' ? 64u : 0u) | ((ch == 'G' || ch == 'H') ? 128u : 0u);
        };
        for (int row = 0; row < n; ++row)
            for (int col = 0; col < n; ++col)
                for (int a = 0; a < 4; ++a) {
                    const int s = row * n + col;
                    const char ch = map[row][col];
                    uint32_t w;
                    if (ch == 'G' || ch == 'H') w = (uint32_t)s | 128u;              // (1.0, s, 0, true)
                    else if (c.slippery)                                             // [(a-1)%4, a, (a+1)%4]
                        w = outcome(row, col, (a + 3) & 3) | (outcome(row, col, a) << 8) |
                            (outcome(row, col, (a + 1) & 3) << 16) | (1u << 24);
                    else w = outcome(row, col, a);
                    e.trans[s * 4 + a] = w;
                }
        e.slippery = c.slippery ? 1 : 0;
        const double third = 1.0 / 3.0;
        e.th1 = 0.0 + third;
        e.th2 = e.th1 + third;
        e.th3 = e.th2 + third;
        e.trunc_reward = edited ? -1.0 : 0.0;   // frozen_lake.rs:119-122 / frozen_lake_edited.rs:227-231
    } else if (c.kind == RL_ENV_CLIFF_WALKING) {
        e.S = 48;
        e.A = 4;
        e.trans.assign(48 * 4, 0);
        for (int row = 0; row < 4; ++row)
            for (int col = 0; col < 12; ++col)
                for (int a = 0; a < 4; ++a) {
                    int nr, nc;
                    grid_move(4, 12, row, col, a, nr, nc);
                    const int ns = nr * 12 + nc;
                    const bool cliff = ns >= 37 && ns <= 46, goal = ns == 47;  // cliff_walking.rs:9-11
                    e.trans[(row * 12 + col) * 4 + a] =
                        (uint32_t)ns | (cliff ? 64u : 0u) | ((cliff || goal) ? 128u : 0u);
                }
        e.start.assign(48, 0.0);
        e.start[36] = 1.0;
        e.trunc_reward = -100.0;
    } else if (c.kind == RL_ENV_TAXI) {
        e.S = 500;
        e.A = 6;
        e.trans.assign(500 * 6, 0);
        e.start.assign(500, 0.0);
        double total = 0.0;
        auto enc = [](int r, int cc, int p, int d) { return ((r * 5 + cc) * 5 + p) * 4 + d; };
        for (int r = 0; r < 5; ++r)
            for (int cc = 0; cc < 5; ++cc)
                for (int p = 0; p < 5; ++p)
                    for (int d = 0; d < 4; ++d) {
                        const int s = enc(r, cc, p, d);
                        if (p < 4 && p != d) { e.start[s] += 1.0; total += 1.0; }
                        for (int a = 0; a < 6; ++a) {
                            int nr = r, nc = cc, np = p;
                            uint32_t rcode = 0;  // -1
                            bool term = false;
                            if (a == 0) nr = std::min(r + 1, 4);
                            else if (a == 1) nr = std::max(r - 1, 0);
                            if (a == 2 && kTaxiMap[1 + r][2 * cc + 2] == ':') nc = std::min(cc + 1, 4);
                            else if (a == 3 && kTaxiMap[1 + r][2 * cc] == ':') nc = std::max(cc - 1, 0);
                            else if (a == 4) {
                                if (p < 4 && r == kTaxiLocs[p][0] && cc == kTaxiLocs[p][1]) np = 4;
                                else rcode = 1;  // -10
                            } else if (a == 5) {
                                if (r == kTaxiLocs[d][0] && cc == kTaxiLocs[d][1] && p == 4) {
                                    np = d; term = true; rcode = 2;  // +20
                                } else rcode = 1;
                            }
                            e.trans[s * 6 + a] = (uint32_t)enc(nr, nc, np, d) | (rcode << 9) | ((term ? 1u : 0u) << 11);
                        }
                    }
        for (double &v : e.start) v /= total;   // taxi.rs:117-119
        e.trunc_reward = 0.0;
        // the kernels compute Taxi's transitions (rl_taxi.h taxi_word): all 3000 must
        // equal the table built above
        for (uint32_t i = 0; i < 500u * 6u; ++i)
            if (taxi_word(i / 6u, i % 6u) != e.trans[i]) return fail(RL_E_STATE, "taxi_word differs from the table");
    } else if (c.kind == RL_ENV_BLACKJACK) {
        e.S = 32 * 32 * 2;   // dense (p_score <= 31, d_score <= 26 in 5 bits, p_ace): (p*32 + d)*2 + ace
        e.A = 2;
    } else {
        return fail(RL_E_ARG, "unknown env kind");
    }
    if (!e.start.empty()) finish_cdf(e);
    if (c.kind == RL_ENV_TAXI && !taxi_start_checked(e)) return fail(RL_E_STATE, "taxi_start differs from categorical_sample");
    // the device FrozenLake resets assume the built-in maps' single start at 0 (rl_device.h)
    if (e.map && e.fixed_start != 0) return fail(RL_E_ARG, "FrozenLake map must start at position 0");
    return RL_OK;
}

// NeuralPolicy input features of every dense state (rl.h rl_input_adapter)
int net_feature_table(const rl_env_config &c, const EnvHost &e, int input, std::vector<double> &feat, uint32_t &n_in) {
    if (input == RL_INPUT_FL_OBS) {
        if (!e.map) return fail(RL_E_ARG, "the FrozenLakeObs adapter needs FrozenLake / FrozenLakeEdited");
        n_in = 6;
        feat.assign((size_t)e.S * 6, 0.0);
        for (uint32_t s = 0; s < e.S; ++s) {
            const int row = (int)s / e.n, col = (int)s % e.n;
            for (int a = 0; a < 4; ++a) feat[s * 6 + a] = terrain_value(neighbour(e.map, e.n, row, col, a));
            feat[s * 6 + 4] = (double)row;
            feat[s * 6 + 5] = (double)col;
        }
        return RL_OK;
    }
    if (input != RL_INPUT_SCALAR) return fail(RL_E_ARG, "unknown input adapter");
    if (c.kind == RL_ENV_FROZEN_LAKE_EDITED)
        return fail(RL_E_ARG, "FrozenLakeEdited observations are FrozenLakeObs structs: use RL_INPUT_FL_OBS");
    n_in = 1;
    feat.assign(e.S, 0.0);
    for (uint32_t s = 0; s < e.S; ++s) feat[s] = (double)rl_obs_to_reference(c.kind, s);   // obs as f64
    return RL_OK;
}
// rand 0.8.5 UniformFloat::<f64>::new(low, high): scale decreased until
// scale * max_rand + low < high
double uniform_scale(double low, double high) {
    const double max_rand = 1.0 - 0x1p-52;
    double scale = high - low;
    while (scale * max_rand + low >= high) {
        uint64_t b;
        std::memcpy(&b, &scale, 8);
        b -= 1;
        std::memcpy(&scale, &b, 8);
    }
    return scale;
}

// value of a fixed-point Q word (matches rlamd::q_val on the device)
double q_value(int64_t raw) { return (double)raw * 0x1p-40; }
uint64_t f64_bits(double x) {
    uint64_t u;
    std::memcpy(&u, &x, 8);
    return u;
}
double f64_of(uint64_t u) {
    double x;
    std::memcpy(&x, &u, 8);
    return x;
}
// NaN stored canonical (rl_device.h canon_nan): equal states compare bitwise
uint64_t canon_bits(double x) { return x != x ? 0x7FF8000000000000ull : f64_bits(x); }
// a value the fixed point holds exactly and within its range
bool fix_exact(double v) {
    if (!(std::fabs(v) <= 2048.0)) return false;
    const double x = v * 0x1p40;
    return x == std::rint(x);
}
// traces grid: every contribution fl(lr * fl(td * E)) of a group step is below
// 2^(max(code(td),1) - 1024 + k) with 2^k >= 4 * |lr| * Ebound * (1 + 2^-50), i.e.
// below 2^51 units of the grid 2^(max(code,1) - 1075 + k): the kernels convert it
// with the 1.5*2^52 magic add (rl_train_impl.h contrib_tr); Ebound
// bounds an accumulating trace (elegibility_traces_agent.rs:75-96: E += 1 on a
// visit, E *= gamma*lambda per sweep).  Same formula as the oracle's
// rlo_trace_grid_k (oracle/rlref.c).
int trace_grid_k(double lr, double gamma, double lambda, uint32_t max_steps, int env) {
    const double gl = gamma * lambda, a = std::fabs(gl);
    double eb;
    if (a < 1.0) {
        eb = 1.0 / (1.0 - a);
    } else {
        // sum_{k=0..T} a^k in closed form (T in 64 bits: max_steps + 1 cannot wrap;
        // O(1)); expm1/log1p keep it accurate for a just above 1, and
        // it is +inf when the sum overflows
        const uint64_t T = env == RL_ENV_BLACKJACK ? 32u : (uint64_t)max_steps + 1u;
        eb = a == 1.0 ? (double)(T + 1u) : std::expm1((double)(T + 1u) * std::log1p(a - 1.0)) / (a - 1.0);
    }
    const double x = std::fabs(lr) * eb * (1.0 + 0x1p-50) * 1.0001;
    if (!(x > 0.0)) return 0;
    if (!(x < INFINITY)) return 1100;
    int ex;
    (void)std::frexp(x, &ex);
    ex += 2;   // two guard bits: |raw| < 2^51
    return ex < -1100 ? -1100 : (ex > 1100 ? 1100 : ex);
}
// merge grid headroom: n values below 2^(53-h) grid units sum below 2^63 for up
// to 2^(10+h) groups (oracle fq_merge_headroom)
int merge_headroom(uint64_t groups) {
    int h = 0;
    while (h < 64 && ((uint64_t)1 << h) < groups) ++h;
    return h - 10 > 0 ? h - 10 : 0;
}

template <class T>
int dalloc(T **p, size_t n) {
    *p = nullptr;
    if (n == 0) return RL_OK;
    HIPC(hipMalloc((void **)p, n * sizeof(T)));
    return RL_OK;
}
template <class T>
void dfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

}  // namespace

#define NCCLC(expr)                                                                                \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess) return fail(RL_E_RCCL, std::string(#expr) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// ====================================================================== handles
// One RCCL communicator per process (one GPU per rank): the only
// collective of the path is the int64 sum of the merge delta over xGMI.
struct rl_comm {
    ncclComm_t comm = nullptr;
    int32_t rank = 0, world = 1, device = 0;
    int64_t *word = nullptr;   // one device int64 for the done-lane agreement of train()/evaluate()
    // host-value all-reduces (rl_comm_allreduce_f64: the bench's barrier and max time)
    hipStream_t stream = nullptr;
    double *vals = nullptr;
    uint32_t n_vals = 0;
};
struct rl_env {
    rl_env_config cfg{};
    EnvHost eh;
    int device = 0;
    hipStream_t stream = nullptr;
    // an Env view of an agent's lanes (rl_agent_env): lane records, RNG streams and
    // tables are the agent's, calls run on the agent's stream
    bool view = false;
    rl_agent *owner = nullptr;
    uint32_t L = 0;
    uint4 *core = nullptr, *rng = nullptr;
    uint32_t *trans = nullptr;
    double *cdf = nullptr;
    uint32_t *act_d = nullptr;
    uint64_t *obs_d = nullptr;
    double *rew_d = nullptr;
    uint8_t *term_d = nullptr;
    std::vector<uint8_t> ready;
    // a view's lanes moved under it (a train launch of its agent): ready is re-read
    // from the lane records (LF_READY) before the next call uses it
    bool ready_stale = false;
    KParams kp{};
};

struct rl_agent {
    rl_agent_config cfg{};
    EnvHost eh;
    int device = 0;
    hipStream_t own_stream = nullptr, stream = nullptr;
    uint32_t S = 0, A = 0, P = 1, L = 0, G = 1, K = 1;
    bool priv = false;
    // lanes
    uint4 *core = nullptr, *rng = nullptr, *aux = nullptr;
    double *epi_reward = nullptr;
    // shared
    int64_t *q_base = nullptr;   // fixed-point words or f64 bits (qrepr)
    uint64_t *n_base = nullptr;
    uint64_t *t_base = nullptr;
    // merge buffer [MAX words][SUM words] (merge_layout), own or the caller's:
    // delta_cap words at delta_max, delta = delta_max + the MAX words
    int64_t *delta_own = nullptr, *delta_max = nullptr, *delta = nullptr, *delta_rep = nullptr;
    uint64_t delta_words = 0;    // replica stride: the dense SUM layout
    uint64_t delta_cap = 0;
    bool merge_groups_set = false;   // rl_agent_set_merge_groups / set_comm declared the total
    uint32_t n_rep = 1;
    uint64_t *qslot = nullptr;   // f64 merge: every group's final Q [n_groups][psal]
    uint32_t n_groups = 0, psal = 0;
    uint64_t merge_groups = 0;   // learner groups over every rank
    int qrepr = RL_QREPR_FIXED40;
    int q_forced = 0;            // rl_agent_set_q_mode(RL_QMODE_F64)
    // private
    double *q_priv = nullptr;
    uint64_t *n_priv = nullptr;
    uint64_t *t_priv = nullptr;
    // traces
    double *trace = nullptr;
    uint16_t *tlist = nullptr, *slot_of = nullptr;
    uint32_t *tcnt = nullptr, *vbits = nullptr;
    size_t vbits_words = 0;
    int trace_layout = -1;   // layout_sparse_traces() of the kernel the trace sets were built for
    // Dyna model (private mode)
    uint32_t plan = 0;
    uint32_t *mcnt = nullptr, *mslot = nullptr;
    uint4 *mrec = nullptr;
    // NeuralPolicy
    bool neural = false;
    uint32_t n_in = 0, n_params = 0, net_gen = 0xffffffffu;
    double *net_w = nullptr, *feat = nullptr;
    // env tables
    uint32_t *trans = nullptr;
    double *cdf = nullptr;
    // outputs
    unsigned long long *stats_d = nullptr;
    rl_step_record *rec_d = nullptr;
    bool recording = false;
    std::vector<rl_step_record> rec_h;
    rl_episode_record *elog_d = nullptr;   // episode log ring [cap][L]
    uint32_t *elog_cnt_d = nullptr;
    uint32_t elog_cap = 0;
    uint64_t launches = 0;
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    // train()/evaluate() loop control (k_ctl_word): device {done, lanes, status},
    // two pinned host slots and their events (read one launch behind)
    int64_t *ctl_d = nullptr, *ctl_h = nullptr;
    hipEvent_t ctl_ev[2] = {nullptr, nullptr};
    KParams kp{};
    // per-call Agent surface (rl_agent_get_action / rl_agent_update): device
    // arrays of L entries and their pinned host staging
    unsigned char *call_d = nullptr, *call_h = nullptr;
    rl_env *env_view = nullptr;
    train_launch_fn fn = nullptr;
    dim3 grid, block;
    size_t smem = 0;
    // shared mode: the LDS carve per kernel family (index KParams::episodic: 0 the
    // throughput kernel of rl_agent_run, 1 the episodic one of train / evaluate),
    // whose register-limited residencies differ; the launch takes its own
    size_t smem_v[2] = {0, 0};
    uint32_t trc_kb_v[2] = {0, 0};
    // pair-trace LDS slots per lane of the last launch (PairCache::cap; UINT32_MAX
    // before the first): a launch with another cap re-indexes the HBM slots first
    uint32_t pair_cap_last = UINT32_MAX;
    rl_comm *comm = nullptr;   // multi-GPU: the merge delta is all-reduced over it
    // the one-shot peer-read merge (rl.h ABI 7, rl_misc.hip k_peer_reduce): this
    // rank's IPC-exported exchange region and every rank's mapping of it
    struct PeerMerge {
        int64_t *region = nullptr;           // [2 slots][cap] words, then the epoch flag
        uint64_t cap = 0;                    // words per slot
        int32_t rank = 0, world = 1;
        std::vector<int64_t *> bases;        // rank order; the peers' are IPC mappings
        int64_t **bases_d = nullptr;
        uint32_t *err_d = nullptr;           // a wait that timed out
        int64_t epoch = 0;                   // merges made (every rank makes the same)
        int64_t timeout_ticks = 0;           // wall-clock ticks a rank waits for a peer
        bool on = false;
    } peer;
    double q_abs0 = 0.0;       // shared mode: max |Q| the table was last reset / set to (delta_bound's Q0)
};

namespace {

void agent_sync_params(rl_agent *a);
// the peer-read merge's region handling (defined with the ABI 7 calls below)
int peer_alloc(rl_agent *a);
void peer_detach(rl_agent *a);
void peer_free(rl_agent *a);
int peer_check(rl_agent *a);
int peer_selftest(rl_agent *a, bool *ok);

int agent_select_kernel(rl_agent *a) {
    a->fn = lookup_train(a->cfg.env.kind, a->cfg.agent, a->cfg.policy, a->cfg.selector, a->cfg.algo,
                         a->priv ? 1 : 0);
    if (!a->fn) return fail(RL_E_ARG, "no kernel for this (env, agent, policy, selector)");
    if (!a->priv && a->cfg.selector == RL_SEL_UCB && a->cfg.algo == RL_ALGO_EXPECTED_SARSA &&
        (uint64_t)a->G * a->K >= (1ull << 32))   // a launch's counter increments are u32 per entry
        return fail(RL_E_ARG, "UCB + expected SARSA: group_size * sync_every must stay below 2^32");
    if (a->priv) {
        a->block = dim3(256);
        a->grid = dim3((a->L + 255) / 256);
        a->smem = private_smem_bytes(a->cfg.env.kind, a->cfg.agent, a->cfg.policy, a->cfg.selector, a->S,
                                     a->A, (uint32_t)a->eh.cdf.size());
        // small tables (FrozenLake, CliffWalking; single or double): the launch's
        // lanes keep their Q in LDS (k_train_private_lds), 4 waves of priv_lpw lanes
        // per block (8: 32 lanes, 50 KB for CliffWalking, 3 blocks per CU); slots of
        // P*S*A + 2 f64.  RLAMD_PRIV_LPW = 0 / 2 / 4 / 8 / 16 / 32 / 64 overrides (0: Q in HBM)
        a->kp.priv_lpw = 0;
        const int ek = a->cfg.env.kind;
        // (a NeuralPolicy's parameters in LDS measured 2x SLOWER than its coalesced
        // HBM stream at 16 lanes per wave — the forward / backward passes are VALU work
        // that idle lanes waste: cfg 6 219 against 102 ms per launch, so not for it)
        const uint64_t psa = (uint64_t)a->P * a->S * a->A;
        uint32_t lpw = (!a->neural && psa * 8 <= 4096 &&
                        (ek == RL_ENV_FROZEN_LAKE || ek == RL_ENV_CLIFF_WALKING || ek == RL_ENV_FROZEN_LAKE_EDITED))
                           ? 8u : 0u;
        if (const char *e = getenv("RLAMD_PRIV_LPW")) {
            const uint32_t v = (uint32_t)atoi(e);
            if (v == 0 || v == 2 || v == 4 || v == 8 || v == 16 || v == 32 || v == 64) lpw = lpw ? v : 0u;
        }
        // the bin's network (frozen_lake_neural.rs:130-134) on one-step agents: the
        // lane's parameters in registers for the launch (k_train_private_net);
        // RLAMD_NET_REGS=0 keeps them in HBM (experiments)
        a->kp.net_regs = 0;
        if (a->neural && a->cfg.agent == RL_AGENT_ONE_STEP && a->A == 4 && a->n_in == 1 &&
            a->cfg.net.hidden == 32 && a->cfg.net.act_hidden == RL_ACT_LEAKY_RELU6 &&
            a->cfg.net.act_out == RL_ACT_LINEAR && ek == RL_ENV_FROZEN_LAKE) {
            const char *e = getenv("RLAMD_NET_REGS");
            a->kp.net_regs = (e && atoi(e) == 0) ? 0u : 1u;
        }
        uint32_t pwv = 4;   // waves per block (RLAMD_PRIV_WAVES = 1 / 2 / 4: experiments)
        if (const char *e = getenv("RLAMD_PRIV_WAVES")) {
            const uint32_t v = (uint32_t)atoi(e);
            if (v == 1 || v == 2 || v == 4) pwv = v;
        }
        if (lpw) {
            const uint32_t nl = pwv * lpw;
            const size_t smem = ((a->smem + 15) & ~(size_t)15) + (size_t)nl * (psa + 2) * 8;
            if (smem <= 160 * 1024) {
                a->kp.priv_lpw = lpw;
                a->block = dim3(64 * pwv);
                a->grid = dim3((a->L + nl - 1) / nl);
                a->smem = smem;
            }
        }
    } else {
        a->kp.ucb_pack = (uint64_t)a->G * a->K < 65536ull ? 1 : 0;   // UCB + expected SARSA counters (KParams)
        const uint32_t g = std::min(a->G, a->L);
        // lanes per wave (rl_kparams.h KParams::lpw): 64, or 32 for the pair-pool
        // traces kernel (small tables) when the lanes give fewer than 4 waves per
        // SIMD at 64: the pool sweep is latency-bound and a wave sweeps its lanes'
        // pool 64 items a round whatever its lane count, so half-full waves double
        // the waves hiding latency for the same sweep work (cfg 4, 2^17 lanes: 2 ->
        // 4 waves per SIMD, 0.612 -> 0.536 ms per launch, A/B on one box; 16 lanes
        // per wave measured 0.58x: VGPRs then allow one group per CU).  RLAMD_LPW
        // = 16 / 32 / 64 overrides (experiments)
        uint32_t lpw = 64;
        {
            const int ek = a->cfg.env.kind;
            const bool pool = a->cfg.agent == RL_AGENT_TRACES && a->cfg.policy != RL_POLICY_NEURAL &&
                              !(a->cfg.selector == RL_SEL_UCB && a->cfg.algo == RL_ALGO_EXPECTED_SARSA) &&
                              (ek == RL_ENV_CLIFF_WALKING || ek == RL_ENV_FROZEN_LAKE ||
                               ek == RL_ENV_FROZEN_LAKE_EDITED);
            int ncu = 256;
            (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, a->device);
            if (pool && ((uint64_t)a->L + 63u) / 64u < 16ull * (uint64_t)ncu) lpw = 32;
        }
        if (const char *e = getenv("RLAMD_LPW")) {
            const uint32_t v = (uint32_t)atoi(e);
            if (v == 16 || v == 32 || v == 64) lpw = v;
        }
        while ((g + lpw - 1) / lpw > 16) lpw *= 2;   // <= 1024 threads per block
        a->kp.lpw = lpw;
        a->block = dim3(((g + lpw - 1) / lpw) * 64);
        a->grid = dim3((a->L + a->G - 1) / a->G);
        // pair-trace slots in LDS: what the groups that must be resident together
        // (groups per CU, at most 2048 threads) leave of the 160 KiB, capped at 64
        // KiB (cfg 4, 2^17 lanes in groups of 256: 2 per CU -> 25 slots per lane).
        // Long episodes spill past the slots into HBM, and a wave waits for its
        // longest list, so more slots pay while occupancy holds: measured on cfg 4
        // 16 slots 6.6e9, 25 slots 7.0e9 env-steps/s; 1 group per CU 3.9e9.
        // RLAMD_TRC_KB overrides (experiments)
        {
            int ncu = 256;
            (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, a->device);
            const uint64_t groups = a->grid.x, per_cu = (groups + (uint64_t)ncu - 1) / (uint64_t)ncu;
            const size_t base = shared_smem_bytes(a->cfg.env.kind, a->cfg.agent, a->cfg.policy, a->cfg.selector,
                                                  a->cfg.algo, a->S, a->A, (uint32_t)a->eh.cdf.size(), a->block.x, 0,
                                                  a->qrepr == RL_QREPR_F64, a->kp.ucb_pack);
            // the groups that can be resident at all: the kernel's register-limited
            // occupancy (without the pair slots), not only the 32-wave cap — cfg 4 at
            // 2^19 lanes on one GPU runs 4 groups per CU (128 VGPRs), so each may
            // take 40 KiB, not 20 (2.12e10 -> 2.2e10 env-steps/s measured)
            // The throughput kernel (episodic 0: rl_agent_run) and the episodic one
            // (train / evaluate) differ in register use, so each gets the carve of
            // its own residency (the query once named whichever kernel
            // the previous call had left in KParams::episodic); launch_train_kernel
            // takes the one it launches.  The pair pools / caches move between LDS
            // and HBM at every launch boundary, so the slot count may differ.
            agent_sync_params(a);   // the kernel the query names follows KParams::fq
            const int32_t epi_saved = a->kp.episodic;
            for (int32_t epi = 0; epi < 2; ++epi) {
                a->kp.episodic = epi;
                int occ_regs = 0;
                if (a->fn(a->kp, a->grid, a->block, base, a->stream, &occ_regs) != hipSuccess || occ_regs <= 0)
                    occ_regs = (int)(2048 / a->block.x);
                const uint64_t resident = std::max<uint64_t>(
                    1, std::min<uint64_t>(per_cu, std::min<uint64_t>((uint64_t)occ_regs, 2048 / a->block.x)));
                const int64_t room = (int64_t)(160 * 1024 / resident) - (int64_t)base - 1024;
                a->trc_kb_v[epi] = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(64, room / 1024));
            }
            a->kp.episodic = epi_saved;
        }
        for (int epi = 0; epi < 2; ++epi) {
            if (const char *e = getenv("RLAMD_TRC_KB")) {
                const int v = atoi(e);
                if (v >= 0 && v <= 150) a->trc_kb_v[epi] = (uint32_t)v;
            }
            a->smem_v[epi] = shared_smem_bytes(a->cfg.env.kind, a->cfg.agent, a->cfg.policy, a->cfg.selector,
                                               a->cfg.algo, a->S, a->A, (uint32_t)a->eh.cdf.size(), a->block.x,
                                               a->trc_kb_v[epi], a->qrepr == RL_QREPR_F64, a->kp.ucb_pack);
            if (a->smem_v[epi] > 160 * 1024) return fail(RL_E_ARG, "learner-group tables exceed the 160 KiB LDS");
        }
        const int ep = a->kp.episodic ? 1 : 0;
        a->kp.trc_kb = a->trc_kb_v[ep];
        a->smem = a->smem_v[ep];
    }
    if (a->tcnt) {
        // the trace sets' layout follows the kernel (rl_kparams.h); switching between
        // the pair and the whole-row layout restarts them (empty sets)
        const int lay = layout_sparse_traces(a->cfg.agent, a->cfg.selector, a->cfg.algo, a->priv) ? 1 : 0;
        if (a->trace_layout >= 0 && lay != a->trace_layout) {
            HIPC(hipSetDevice(a->device));
            HIPC(hipMemsetAsync(a->tcnt, 0, (size_t)a->L * 4, a->stream));
            if (a->vbits) HIPC(hipMemsetAsync(a->vbits, 0, a->vbits_words * 4, a->stream));
        }
        a->trace_layout = lay;
    }
    return RL_OK;
}

void bj_term_scan(rl_agent *a, const int64_t *q);
double delta_bound(const rl_agent *a);
int agent_store_table(rl_agent *a, const double *vals);

int agent_reset_policy(rl_agent *a) {
    const size_t PSA = (size_t)a->P * a->S * a->A, SA = (size_t)a->S * a->A;
    if (a->neural) {   // NeuralPolicy::new (generation 0) / Network::reset (src/network.rs:89-93)
        ++a->net_gen;
        const double l1 = std::sqrt(6.0 / (double)(a->n_in + a->cfg.net.hidden));
        const double l2 = std::sqrt(6.0 / (double)(a->cfg.net.hidden + a->A));
        launch_net_init(a->kp, a->cfg.seed, a->cfg.lane_offset, a->net_gen, uniform_scale(-l1, l1), -l1,
                        uniform_scale(-l2, l2), -l2, a->stream);
        HIPC(hipGetLastError());
        HIPC(hipStreamSynchronize(a->stream));
    } else if (a->priv) {
        launch_fill_f64(a->q_priv, PSA * a->L, a->cfg.q_default, a->stream);
        HIPC(hipGetLastError());
        if (a->n_priv) HIPC(hipMemsetAsync(a->n_priv, 0, SA * a->L * 8, a->stream));
        if (a->t_priv) {
            std::vector<uint64_t> ones(a->L, 1);
            HIPC(hipMemcpyAsync(a->t_priv, ones.data(), a->L * 8, hipMemcpyHostToDevice, a->stream));
            HIPC(hipStreamSynchronize(a->stream));
        }
    } else {
        const std::vector<double> v(PSA, a->cfg.q_default);
        return agent_store_table(a, v.data());
    }
    return RL_OK;
}

// Blackjack terminal rows (dense obs with player sum > 21 or dealer card > 10:
// rl_train_impl.h bj_nonterminal) are read-only for the kernels; record whether
// each table holds one word there (KParams::bj_tconst)
void bj_term_scan(rl_agent *a, const int64_t *q) {
    a->kp.bj_tconst = 0;
    if (a->cfg.env.kind != RL_ENV_BLACKJACK || a->priv) return;
    const size_t SA = (size_t)a->S * a->A;
    int64_t v[2] = {0, 0};
    for (uint32_t t = 0; t < a->P; ++t) {
        bool first = true;
        for (uint32_t s = 0; s < a->S; ++s) {
            const uint32_t pl = s >> 6, d = (s >> 1) & 31u;
            if (pl <= 21u && d <= 10u) continue;
            for (uint32_t b = 0; b < a->A; ++b) {
                const size_t i = t * SA + (size_t)s * a->A + b;
                if (first) { v[t] = q[i]; first = false; }
                else if (q[i] != v[t]) return;
            }
        }
    }
    a->kp.bj_tconst = 1;
    a->kp.bj_traw[0] = v[0];
    a->kp.bj_traw[1] = v[1];
}

int agent_reset_selector(rl_agent *a) {
    const size_t SA = (size_t)a->S * a->A;
    if (a->priv) {
        if (a->n_priv) HIPC(hipMemsetAsync(a->n_priv, 0, SA * a->L * 8, a->stream));
        if (a->t_priv) {
            std::vector<uint64_t> ones(a->L, 1);
            HIPC(hipMemcpyAsync(a->t_priv, ones.data(), a->L * 8, hipMemcpyHostToDevice, a->stream));
            HIPC(hipStreamSynchronize(a->stream));
        }
    } else {
        HIPC(hipMemsetAsync(a->n_base, 0, SA * 8, a->stream));
        const uint64_t one = 1;
        HIPC(hipMemcpyAsync(a->t_base, &one, 8, hipMemcpyHostToDevice, a->stream));
        HIPC(hipStreamSynchronize(a->stream));
    }
    launch_arm_full(a->kp, -1, 0, 1, a->cfg.eps0, a->stream);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}

// max |reward| an env step can return, truncation included
double env_reward_bound(int kind) {
    switch (kind) {
    case RL_ENV_FROZEN_LAKE: return 1.0;           // frozen_lake.rs:44 (0/1), :121 (0)
    case RL_ENV_FROZEN_LAKE_EDITED: return 10.0;   // frozen_lake_edited.rs (+10 goal, -1 otherwise)
    case RL_ENV_CLIFF_WALKING: return 100.0;       // cliff_walking.rs (-100 cliff / truncation, -1)
    case RL_ENV_TAXI: return 20.0;                 // taxi.rs:76-110 (+20, -10, -1), truncation 0
    case RL_ENV_BLACKJACK: return 1.0;             // blackjack.rs (+-1, 0)
    default: return std::numeric_limits<double>::infinity();
    }
}

// Can a shared-mode entry reach the |Q| <= 2048 clamp, or a TD delta saturate at
// +-2^51 raw?  Provable only for the one-step agent on a single table: the
// double policy writes one table with a TD error taken on the other
// (double_tabular_policy.rs:31-67: Q_u += lr*(r + gamma*F - Q_v)), and the
// eligibility traces move every visited entry by the CURRENT pair's error
// (elegibility_traces_agent.rs:82-96) — neither update contracts the entry it
// writes (the double policy's A - B grows by (1 + lr) per update pair; cfg 5 clamps
// at bench length), so both are counted, never assumed.  For the one-step
// tabular agent, not when the bootstrap F is a sub-convex combination of Q values —
// SARSA's pick, Q-learning's max, expected SARSA over eps-greedy's probabilities
// (eps/A each and 1-eps at the argmax: non-negative for eps in [0,1], summing to
// 1-eps/A; src/agent.rs:19-45, uniform_epsilon_greed.rs:72-76).  Then one update
// Q' = (1-lr)Q + lr(r + gamma*F) with lr in [0,1] keeps |Q'| <= max(M, R/(1-gamma))
// when |Q|, |F| <= M; a step's mean of such values and the merge's mean over groups
// keep the bound, so by induction every entry stays within Mb = max(|Q_0|,
// R/(1-gamma)), and every delta within lr*(R + (1+gamma)Mb).
// UCB + expected SARSA weighs by u_i / sum(u) (upper_confidence_bound.rs:48-63):
// no bound, its kernels always count.
// Returns the proven bound on |lr * E * td| (+inf when nothing is proven); the
// fixed point (|Q| <= 2048) is used only when it is < 2000 (fix_proven), every
// other table is held in f64 (rl.h rl_q_repr).
double delta_bound(const rl_agent *a) {
    const double inf = std::numeric_limits<double>::infinity();
    const rl_agent_config &c = a->cfg;
    if (a->priv || a->neural) return inf;
    if (c.agent != RL_AGENT_ONE_STEP || c.policy != RL_POLICY_TABULAR) return inf;
    if (c.selector == RL_SEL_UCB && c.algo == RL_ALGO_EXPECTED_SARSA) return inf;
    const double lr = c.lr, g = c.gamma;
    if (!(lr >= 0.0 && g >= 0.0 && g < 1.0 && std::isfinite(a->q_abs0))) return inf;
    const double emax = 1.0;   // one-step: the written entry's own error, weight lr
    if (!(lr * emax <= 1.0)) return inf;
    if (c.selector == RL_SEL_EPS_GREEDY && c.algo == RL_ALGO_EXPECTED_SARSA) {
        // eps stays in [eps_final, eps0] (or decays toward 0 by a factor in [0,1])
        const bool dec = c.decay_kind == RL_DECAY_MUL ? (c.eps_decay >= 0.0 && c.eps_decay <= 1.0) : c.eps_decay >= 0.0;
        if (!(c.eps0 >= 0.0 && c.eps0 <= 1.0 && c.eps_final >= 0.0 && dec)) return inf;
    }
    const double R = env_reward_bound(c.env.kind);
    const double mb = std::max(a->q_abs0, R / (1.0 - g));
    if (!(mb <= 2000.0)) return inf;
    // the kernels that rely on this bound also convert episode rewards (at most
    // max_steps + 1 steps of |r| <= R; Blackjack: one +-1) to 2^-16 fixed point
    // with a rint valid below 2^51
    const double ep_len = c.env.kind == RL_ENV_BLACKJACK ? 1.0 : (double)c.env.max_steps + 1.0;
    if (!(ep_len * R * 65536.0 < 0x1p50)) return inf;
    return lr * emax * (R + (1.0 + g) * mb);
}
// Round 6: on a slippery map the fixed point stays in range
// but not within the north star's 1e-5 of f64.  Its 2^-40 rounding decides greedy
// ties the f64 table breaks the other way, lanes' trajectories part from the
// second launch, and rare transitions then move entries by up to 1.9e-4 (cfg 2
// slippery, tests/golden/longrun.json repr_drift_curve; the deterministic map stays
// below 8.5e-6) — so "auto" keeps slippery FrozenLake tables in f64.  Same rule as
// the oracle's o_proven.
bool fix_faithful(const rl_agent *a) {
    const int k = a->cfg.env.kind;
    return !((k == RL_ENV_FROZEN_LAKE || k == RL_ENV_FROZEN_LAKE_EDITED) && a->cfg.env.slippery);
}
bool fix_proven(const rl_agent *a) { return delta_bound(a) < 2000.0 && fix_faithful(a); }
// The 8-wave kernels pack a step's contributions to an entry into one int64,
// sum * 2^11 + count (one LDS atomic per contribution instead of two): exact
// while at most G contributions of at most delta_bound * 2^40 + 1 raw units each
// keep |sum| * 2^11 + 2047 below 2^63 — and |sum| below 2^51, so the settle converts
// it with the 1.5*2^52 magic add: G * delta_bound < 2^11 (FrozenLake and Blackjack
// at the CLI defaults: 0.15 * 512 and 2.0 * 512)
bool pack_proven(const rl_agent *a) { return (double)a->G * delta_bound(a) < 2000.0; }

// Write a freshly set table (P*S*A values) as the shared base: in the fixed point
// when allowed (not forced to f64, the proof holds with Q0 = max |value|, every
// value exact in it), else as f64 bits (NaN canonical).  Same rule as the
// oracle's o_choose_repr (oracle/rlref.c).
int agent_store_table(rl_agent *a, const double *vals) {
    const size_t PSA = (size_t)a->P * a->S * a->A;
    double amax = 0.0;
    for (size_t i = 0; i < PSA; ++i) {
        const double x = std::fabs(vals[i]);
        amax = x != x ? INFINITY : std::max(amax, x);
    }
    a->q_abs0 = amax;
    bool fix = !a->q_forced && fix_proven(a);
    for (size_t i = 0; fix && i < PSA; ++i) fix = fix_exact(vals[i]);
    std::vector<int64_t> w(PSA);
    for (size_t i = 0; i < PSA; ++i) w[i] = fix ? (int64_t)(vals[i] * 0x1p40) : (int64_t)canon_bits(vals[i]);
    a->qrepr = fix ? RL_QREPR_FIXED40 : RL_QREPR_F64;
    HIPC(hipMemcpyAsync(a->q_base, w.data(), PSA * 8, hipMemcpyHostToDevice, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    bj_term_scan(a, w.data());
    return agent_select_kernel(a);   // the kernel and its LDS carve follow the representation
}
// the base's values as f64 (either representation)
int agent_table_values(rl_agent *a, std::vector<double> &vals, std::vector<int64_t> &w) {
    const size_t PSA = (size_t)a->P * a->S * a->A;
    w.resize(PSA);
    vals.resize(PSA);
    HIPC(hipMemcpyAsync(w.data(), a->q_base, PSA * 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    for (size_t i = 0; i < PSA; ++i)
        vals[i] = a->qrepr == RL_QREPR_F64 ? f64_of((uint64_t)w[i]) : q_value(w[i]);
    return RL_OK;
}
// fixed point -> f64 (exact: |raw| <= 2^51)
int agent_to_f64(rl_agent *a) {
    std::vector<double> v;
    std::vector<int64_t> w;
    int rc = agent_table_values(a, v, w);
    if (rc) return rc;
    for (size_t i = 0; i < w.size(); ++i) w[i] = (int64_t)canon_bits(v[i]);
    HIPC(hipMemcpyAsync(a->q_base, w.data(), w.size() * 8, hipMemcpyHostToDevice, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    a->qrepr = RL_QREPR_F64;
    bj_term_scan(a, w.data());
    return agent_select_kernel(a);
}
// after a selector / algorithm change: a fixed-point table whose proof no longer
// holds continues in f64 (the proof follows the table's real state)
int agent_recheck_repr(rl_agent *a) {
    if (!a->priv && a->qrepr == RL_QREPR_FIXED40 && !fix_proven(a)) return agent_to_f64(a);
    return agent_select_kernel(a);
}

// LDS-held entries per learner group: Blackjack eps-greedy keeps the 484 non-terminal rows
uint32_t lds_entries(const rl_agent *a) {
    return (a->cfg.env.kind == RL_ENV_BLACKJACK && a->cfg.selector != RL_SEL_UCB) ? a->P * 484u * a->A
                                                                                 : a->P * a->S * a->A;
}
// words of the merge buffer the current representation uses (all-reduced):
// f64 MAX [psal] + SUM [psal sums][psal counts][SA dN][1 dt][3 x psal kinds];
// fixed point no MAX words, SUM [PSA dQ][PSA counts][SA dN][1 dt]
void merge_layout(const rl_agent *a, uint64_t *max_words, uint64_t *sum_words) {
    const uint64_t SA = (uint64_t)a->S * a->A, PSA = a->P * SA, ps = lds_entries(a);
    if (a->qrepr == RL_QREPR_F64) { *max_words = ps; *sum_words = 5 * ps + SA + 1; }
    else { *max_words = 0; *sum_words = 2 * PSA + SA + 1; }
}

void agent_sync_params(rl_agent *a) {
    KParams &p = a->kp;
    p.lr = a->cfg.lr;
    p.lr40 = ldexp(a->cfg.lr, 40);
    p.gamma = a->cfg.gamma;
    p.gl = a->cfg.gamma * a->cfg.lambda;   // discount_factor * lambda_factor (elegibility_traces_agent.rs:94)
    p.eps_decay = a->cfg.eps_decay;
    p.eps_final = a->cfg.eps_final;
    p.ucb_c = a->cfg.ucb_c;
    p.decay_kind = a->cfg.decay_kind;
    p.eps_dm = a->cfg.decay_kind == RL_DECAY_MUL ? a->cfg.eps_decay : 1.0;
    p.eps_ds = a->cfg.decay_kind == RL_DECAY_MUL ? 0.0 : a->cfg.eps_decay;
    p.algo = a->cfg.algo;
    p.fq = a->qrepr == RL_QREPR_F64 ? 1 : 0;
    p.pack_ok = !p.fq && pack_proven(a) ? 1 : 0;
    p.trace_k = trace_grid_k(a->cfg.lr, a->cfg.gamma, a->cfg.lambda, a->cfg.env.max_steps, a->cfg.env.kind);
    p.merge_hb = merge_headroom(a->merge_groups);
    if (!a->priv) {
        uint64_t mw, sw;
        merge_layout(a, &mw, &sw);
        a->delta = a->delta_max + mw;
        p.sum_words = (uint32_t)sw;
    }
    p.delta = a->delta;
    p.delta_max = a->delta_max;
    p.qslot = a->qslot;
    p.n_groups = a->n_groups;
    p.psal = lds_entries(a);
    p.plan_steps = a->plan;
    p.mcnt = a->mcnt; p.mrec = a->mrec; p.mslot = a->mslot;
    p.elog = a->elog_cap ? a->elog_d : nullptr;
    p.elog_cnt = a->elog_cnt_d;
    p.elog_cap = a->elog_cap;
}

// merge != nullptr: the caller applies the merge right after this launch (one
// process, its own delta); *merge = true when the fused fold + apply did it
int launch_train_kernel(rl_agent *a, bool *merge = nullptr) {
    agent_sync_params(a);
    if (!a->priv) {
        uint64_t mw, sw;
        merge_layout(a, &mw, &sw);
        if (mw + sw > a->delta_cap)
            return fail(RL_E_STATE, "merge buffer smaller than the current Q representation needs "
                                    "(rl_agent_delta_words): set a larger one");
    }
    a->kp.episodic = (a->kp.target_episodes || a->kp.eval_at || a->kp.eval_only) ? 1 : 0;
    if (!a->priv) {   // the LDS carve of the kernel family this launch takes (agent_select_kernel)
        a->kp.trc_kb = a->trc_kb_v[a->kp.episodic];
        a->smem = a->smem_v[a->kp.episodic];
    }
    // the pair lists' LDS slot count follows the carve, which differs
    // between the kernel families and changes with the selector / representation,
    // while a lane's list survives the launch boundary (p.tcnt).  The HBM slots'
    // index (slot_of) and visited-state bitmap (vbits) are kept only for slots >=
    // cap, so a launch with another cap rebuilds them for its own first
    if (!a->priv && a->vbits && a->tcnt && pair_slot_index_env(a->cfg.env.kind) &&
        layout_sparse_traces(a->cfg.agent, a->cfg.selector, a->cfg.algo, 0)) {
        const uint32_t cap = shared_pair_cap(a->cfg.env.kind, a->cfg.agent, a->cfg.policy, a->cfg.selector,
                                             a->cfg.algo, a->S, a->A, (uint32_t)a->eh.cdf.size(), a->block.x,
                                             a->kp.trc_kb, a->qrepr == RL_QREPR_F64, a->kp.ucb_pack);
        if (a->pair_cap_last != UINT32_MAX && cap != a->pair_cap_last) {
            launch_pair_reindex(a->kp, cap, a->stream);
            HIPC(hipGetLastError());
        }
        a->pair_cap_last = cap;
    }
    if (a->recording) a->kp.rec = a->rec_d; else a->kp.rec = nullptr;
    // the launch moves the lanes an Env view shares: a lane the view
    // once reset may have terminated since (the reference's Err(EnvNotReady),
    // src/env.rs:17,24), and one still mid-episode may keep stepping:
    // the view re-reads each lane's LF_READY after the launch (view_ready_refresh)
    if (a->env_view) a->env_view->ready_stale = true;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (a->timing) {
        HIPC(hipEventCreate(&e0));
        HIPC(hipEventCreate(&e1));
        HIPC(hipEventRecord(e0, a->stream));
    }
    {
        const hipError_t le = a->fn(a->kp, a->grid, a->block, a->smem, a->stream, nullptr);
        if (le != hipSuccess)
            return fail(RL_E_HIP, std::string("train kernel launch (smem ") + std::to_string(a->smem) +
                                      " B, block " + std::to_string(a->block.x) + "): " + hipGetErrorString(le));
    }
    if (a->timing) {
        HIPC(hipEventRecord(e1, a->stream));
        a->events.emplace_back(e0, e1);
    }
    if (merge) *merge = false;
    if (!a->priv) {
        if (a->qrepr == RL_QREPR_F64) {   // f64 merge, first phase (UCB: ΔN / Δt from the replicas)
            if (a->cfg.selector == RL_SEL_UCB) launch_fold_replicas(a->kp, a->stream);
            launch_fq_merge_a(a->kp, a->stream);
        } else if (merge && a->delta_max == a->delta_own && a->cfg.selector != RL_SEL_UCB && !a->comm &&
                   !a->peer.on) {
            launch_fold_apply(a->kp, a->stream);   // fold the replicas and apply (eps-greedy: sums + counts only)
            *merge = true;
        } else if (merge && a->peer.on) {
            // the fixed point over the peers: the replicas folded into this rank's
            // exchange slot, then the ranks' words reduced and applied (two launches)
            auto &pm = a->peer;
            uint64_t mw, sw;
            merge_layout(a, &mw, &sw);
            if (sw > pm.cap) return fail(RL_E_STATE, "merge buffer larger than the peer exchange slots");
            const uint64_t slot = (uint64_t)(pm.epoch & 1) * pm.cap;
            ++pm.epoch;
            launch_peer_fold_put(a->kp, pm.region + slot, a->stream);
            launch_peer_reduce_apply(a->kp, pm.bases_d, (uint32_t)pm.world, (uint32_t)pm.rank, slot,
                                     2 * pm.cap + 16, pm.epoch, pm.err_d, pm.timeout_ticks, a->stream);
            *merge = true;
        } else {
            launch_fold_replicas(a->kp, a->stream);   // fold the group-delta replicas into the delta
        }
        HIPC(hipGetLastError());
    }
    a->launches++;
    if (a->recording) {
        const size_t n = (size_t)a->K * a->L;
        const size_t off = a->rec_h.size();
        a->rec_h.resize(off + n);
        HIPC(hipMemcpyAsync(a->rec_h.data() + off, a->rec_d, n * sizeof(rl_step_record),
                            hipMemcpyDeviceToHost, a->stream));
        HIPC(hipStreamSynchronize(a->stream));
    }
    return RL_OK;
}

// f64 merge, second phase (after the MAX all-reduce): the grid sums; nothing for the fixed point
int launch_fold_kernel(rl_agent *a) {
    if (a->priv || a->qrepr != RL_QREPR_F64) return RL_OK;
    agent_sync_params(a);
    launch_fq_merge_b(a->kp, a->stream);
    HIPC(hipGetLastError());
    return RL_OK;
}
int launch_apply_kernel(rl_agent *a) {
    if (a->priv) return RL_OK;
    agent_sync_params(a);
    if (a->qrepr == RL_QREPR_F64) launch_fq_apply(a->kp, a->stream);
    else launch_apply(a->kp, a->stream);
    HIPC(hipGetLastError());
    return RL_OK;
}

// the merge's collectives, in place on the agent's stream: the MAX words (f64:
// per-entry grid codes) and the SUM words (grid sums / ΔQ, group counts, ΔN, Δt,
// NaN / inf counts) over every rank.  Exact int64 arithmetic, so Q is
// bit-identical for any rank count at a fixed global lane set.
int comm_live(rl_agent *a);
// the peer-read all-reduce of n int64 words of buf, in place on the agent's stream
// (rl.h ABI 7; the protocol is at k_peer_reduce): the words to this rank's slot,
// then one kernel raises its flag, waits for every peer's and reduces in rank order
int peer_allreduce(rl_agent *a, int64_t *buf, uint64_t n, bool op_max) {
    auto &pm = a->peer;
    if (n > pm.cap) return fail(RL_E_STATE, "merge buffer larger than the peer exchange slots");
    const uint64_t slot = (uint64_t)(pm.epoch & 1) * pm.cap;
    ++pm.epoch;
    launch_peer_put(buf, pm.region + slot, n, a->stream);
    launch_peer_reduce(pm.bases_d, (uint32_t)pm.world, (uint32_t)pm.rank, slot, 2 * pm.cap + 16, n, pm.epoch,
                       op_max ? 1 : 0, buf, pm.err_d, pm.timeout_ticks, a->stream);
    HIPC(hipGetLastError());
    return RL_OK;
}
int allreduce_max(rl_agent *a) {
    if ((!a->comm && !a->peer.on) || a->qrepr != RL_QREPR_F64) return RL_OK;
    uint64_t mw, sw;
    merge_layout(a, &mw, &sw);
    if (a->peer.on) return peer_allreduce(a, a->delta_max, mw, true);
    if (int rc = comm_live(a)) return rc;
    NCCLC(ncclAllReduce(a->delta_max, a->delta_max, mw, ncclInt64, ncclMax, a->comm->comm, a->stream));
    return RL_OK;
}
int allreduce_delta(rl_agent *a) {
    if (!a->comm && !a->peer.on) return RL_OK;   // no communicator: this process's delta is the total
    uint64_t mw, sw;
    merge_layout(a, &mw, &sw);
    if (a->peer.on) return peer_allreduce(a, a->delta, sw, false);
    if (int rc = comm_live(a)) return rc;
    NCCLC(ncclAllReduce(a->delta, a->delta, sw, ncclInt64, ncclSum, a->comm->comm, a->stream));
    return RL_OK;
}
// the merge after a launch: [MAX] -> fold -> [SUM] -> apply
int merge_after_launch(rl_agent *a) {
    int rc;
    if ((rc = allreduce_max(a)) || (rc = launch_fold_kernel(a)) || (rc = allreduce_delta(a))) return rc;
    return launch_apply_kernel(a);
}
// one launch of K steps + the merge (fused fold+apply for a one-process eps-greedy learner)
int launch_and_merge(rl_agent *a) {
    bool merged = false;
    int rc = launch_train_kernel(a, &merged);
    if (rc) return rc;
    if (merged) return RL_OK;
    return merge_after_launch(a);
}
// sum of a host value over the ranks (1 rank: itself)
int comm_live(rl_agent *a) {
    if (a->comm && !a->comm->comm) return fail(RL_E_STATE, "communicator aborted after a fatal error on this rank");
    return RL_OK;
}
int allreduce_u64(rl_agent *a, uint64_t v, uint64_t *sum) {
    *sum = v;
    if (!a->comm) return RL_OK;
    if (int rc = comm_live(a)) return rc;
    int64_t x = (int64_t)v;
    HIPC(hipMemcpyAsync(a->comm->word, &x, 8, hipMemcpyHostToDevice, a->stream));
    if (a->peer.on) {
        if (int rc = peer_allreduce(a, a->comm->word, 1, false)) return rc;
    } else {
        NCCLC(ncclAllReduce(a->comm->word, a->comm->word, 1, ncclInt64, ncclSum, a->comm->comm, a->stream));
    }
    HIPC(hipMemcpyAsync(&x, a->comm->word, 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    *sum = (uint64_t)x;
    return RL_OK;
}
// A rank that fails inside the loop cannot join the next collective: abort its
// communicator so the peers' RCCL calls fail instead of waiting on it
int abort_comm(rl_agent *a, int rc) {
    if (a->comm && a->comm->comm) {
        (void)ncclCommAbort(a->comm->comm);
        a->comm->comm = nullptr;
    }
    return rc;
}

enum { CTL_OK = 0, CTL_LAUNCH_CAP = 1, CTL_RECORD_CAP = 2 };

// train() / evaluate(): launch until every lane of every rank is DONE.
// After each launch a one-block kernel forms the control word {lanes DONE, lanes,
// status} (k_ctl_word), one 24-byte all-reduce sums it over the ranks and it is
// copied to pinned host memory.  The host reads launch k's word only after
// queueing launch k + 1, so the loop never drains the stream: the GPU runs one
// launch ahead of the exit test.  That launch is a no-op (DONE lanes draw, update
// and count nothing; an unchanged merge applies zero) except for the step records,
// so a recording agent reads each word right away.  Every rank reads the same
// summed word, so all ranks run the same launches and leave together, also on a
// per-rank condition (the launch cap, the 4 GiB record cap), which travels in the
// status word.  A HIP / RCCL error aborts the communicator (abort_comm).
int run_until_done(rl_agent *a, rl_stats *out) {
    // a lane needs at most (max_steps + 1) steps per episode, so a call that has
    // not finished after this many launches is a bug, not a long run
    const uint64_t max_launches = 1ull << 22;
    const bool dump = getenv("RLAMD_DEBUG_LANES") != nullptr;
    const uint64_t lag = (a->recording || dump) ? 0 : 1;
    int rc = comm_live(a);
    if (rc) return rc;
    rl_stats st0{};
    if ((rc = rl_agent_stats(a, &st0))) return rc;
    for (uint64_t launch = 0;; ++launch) {
        int64_t status = CTL_OK;
        if (launch + 1 >= max_launches) status = CTL_LAUNCH_CAP;
        if ((a->rec_h.size() + (size_t)a->K * a->L) * sizeof(rl_step_record) > (1ull << 32)) status = CTL_RECORD_CAP;
        // done-lane counter (slot 5 of every stats replica) is per launch
        if (hipMemset2DAsync(&a->stats_d[5], STATS_W * 8, 0, 8, STATS_REP, a->stream) != hipSuccess)
            return abort_comm(a, fail(RL_E_HIP, "stats reset"));
        if ((rc = launch_and_merge(a))) return abort_comm(a, rc);
        launch_ctl_word(a->kp, a->ctl_d, a->L, status, a->stream);
        if (hipGetLastError() != hipSuccess) return abort_comm(a, fail(RL_E_HIP, "control word launch"));
        if (a->peer.on) {
            if ((rc = peer_allreduce(a, a->ctl_d, 3, false))) return abort_comm(a, rc);
        } else if (a->comm) {
            const ncclResult_t nr = ncclAllReduce(a->ctl_d, a->ctl_d, 3, ncclInt64, ncclSum, a->comm->comm, a->stream);
            if (nr != ncclSuccess) return abort_comm(a, fail(RL_E_RCCL, std::string("control all-reduce: ") +
                                                                          ncclGetErrorString(nr)));
        }
        const uint32_t slot = (uint32_t)(launch & 1u);
        if (hipMemcpyAsync(a->ctl_h + 3 * slot, a->ctl_d, 24, hipMemcpyDeviceToHost, a->stream) != hipSuccess ||
            hipEventRecord(a->ctl_ev[slot], a->stream) != hipSuccess)
            return abort_comm(a, fail(RL_E_HIP, "control word copy"));
        if (dump) {   // diagnostics: raw lane records per launch
            std::vector<uint4> c(a->L);
            HIPC(hipMemcpy(c.data(), a->core, a->L * 16, hipMemcpyDeviceToHost));
            if (FILE *f = fopen(getenv("RLAMD_DEBUG_LANES"), "ab")) { fwrite(c.data(), 16, a->L, f); fclose(f); }
        }
        if (launch < lag) continue;
        const uint32_t rs = (uint32_t)((launch - lag) & 1u);
        if (hipEventSynchronize(a->ctl_ev[rs]) != hipSuccess) return abort_comm(a, fail(RL_E_HIP, "control word wait"));
        const int64_t *w = a->ctl_h + 3 * rs;
        if (w[2] != CTL_OK) {   // some rank hit a cap: every rank stops here
            HIPC(hipStreamSynchronize(a->stream));
            return fail(RL_E_STATE, w[2] % 2 ? "train/evaluate did not finish (launch cap)"
                                             : "recorded stream exceeds 4 GiB on some rank: record fewer steps");
        }
        if (w[0] >= w[1]) break;
    }
    HIPC(hipStreamSynchronize(a->stream));
    rl_stats st1{};
    if ((rc = rl_agent_stats(a, &st1))) return rc;
    if (st1.delta_saturations != st0.delta_saturations)
        return fail(RL_E_STATE, "f64 merge over more learner groups than its headroom allows "
                                "(rl_agent_set_merge_groups): Q is not the exact mean");
    if (out) *out = st1;
    return RL_OK;
}

}  // namespace

// ====================================================================== C ABI
extern "C" {

const char *rl_last_error(void) { return g_err.c_str(); }
int rl_abi_version(void) { return RL_ABI_VERSION; }
#ifndef RLAMD_BUILD_FLAGS
#define RLAMD_BUILD_FLAGS "unknown"
#endif
#define RLAMD_STR2(x) #x
#define RLAMD_STR(x) RLAMD_STR2(x)
const char *rl_build_info(void) {
    static const std::string s = std::string("librlamd abi " RLAMD_STR(RL_ABI_VERSION) "; target gfx950; RLAMD_EXP="
                                             RLAMD_STR(RLAMD_EXP) "; flags: " RLAMD_BUILD_FLAGS "; id: ") +
                                 rl_build_id();
    return s.c_str();
}
int rl_device_count(int *count) {
    HIPC(hipGetDeviceCount(count));
    return RL_OK;
}

uint64_t rl_blackjack_obs_id(uint32_t p, uint32_t d, uint32_t ace) {
    // fxhash 0.2.1: FxHasher64::write_u8 per field of #[derive(Hash)]
    const uint64_t K = 0x517cc1b727220a95ull;
    uint64_t h = 0;
    const uint64_t w[3] = {p & 0xffu, d & 0xffu, ace ? 1u : 0u};
    for (uint64_t x : w) h = (((h << 5) | (h >> 59)) ^ x) * K;
    return h;
}
uint64_t rl_obs_to_reference(int32_t env_kind, uint32_t s) {
    if (env_kind == RL_ENV_BLACKJACK) return rl_blackjack_obs_id(s >> 6, (s >> 1) & 31u, s & 1u);
    return s;
}
int rl_obs_from_reference(int32_t env_kind, uint64_t obs, uint32_t *dense_state) {
    if (!dense_state) return fail(RL_E_ARG, "null argument");
    if (env_kind != RL_ENV_BLACKJACK) {
        if (obs > 0xffffffffull) return fail(RL_E_ARG, "observation out of range");
        *dense_state = (uint32_t)obs;
        return RL_OK;
    }
    // the 2048 dense Blackjack observations by their fxhash ids (distinct: checked once)
    static const std::vector<std::pair<uint64_t, uint32_t>> ids = [] {
        std::vector<std::pair<uint64_t, uint32_t>> v(2048);
        for (uint32_t s = 0; s < 2048; ++s) v[s] = {rl_obs_to_reference(RL_ENV_BLACKJACK, s), s};
        std::sort(v.begin(), v.end());
        return v;
    }();
    const auto it = std::lower_bound(ids.begin(), ids.end(), std::make_pair(obs, 0u));
    if (it == ids.end() || it->first != obs) return fail(RL_E_ARG, "not a Blackjack observation id");
    *dense_state = it->second;
    return RL_OK;
}

int rl_env_dims(const rl_env_config *cfg, uint32_t *S, uint32_t *A) {
    if (!cfg || !S || !A) return fail(RL_E_ARG, "null argument");
    EnvHost e;
    int rc = build_env(*cfg, e);
    if (rc) return rc;
    *S = e.S;
    *A = e.A;
    return RL_OK;
}

int rl_env_table(const rl_env_config *cfg, double *prob, uint32_t *next, double *reward, uint8_t *term,
                 double *start) {
    if (!cfg) return fail(RL_E_ARG, "null config");
    EnvHost e;
    int rc = build_env(*cfg, e);
    if (rc) return rc;
    if (e.kind == RL_ENV_BLACKJACK) return fail(RL_E_ARG, "Blackjack has no transition table");
    for (uint32_t s = 0; s < e.S; ++s)
        for (uint32_t a = 0; a < e.A; ++a) {
            const uint32_t w = e.trans[s * e.A + a];
            const size_t k = ((size_t)s * e.A + a) * 3;
            double pr[3] = {1.0, 0.0, 0.0};
            uint32_t nx[3] = {0, 0, 0};
            double rw[3] = {0.0, 0.0, 0.0};
            uint8_t tm[3] = {0, 0, 0};
            if (e.kind == RL_ENV_FROZEN_LAKE || e.kind == RL_ENV_FROZEN_LAKE_EDITED) {
                const bool edited = e.kind == RL_ENV_FROZEN_LAKE_EDITED;
                const char cell = e.map[s / e.n][s % e.n];
                const int n = (w >> 24) & 1 ? 3 : 1;
                for (int i = 0; i < n; ++i) {
                    const uint32_t o = (w >> (8 * i)) & 0xffu;
                    pr[i] = n == 3 ? 1.0 / 3.0 : 1.0;
                    nx[i] = o & 63u;
                    rw[i] = edited ? ((o & 64u) ? 10.0 : -1.0) : ((o & 64u) ? 1.0 : 0.0);
                    tm[i] = (o & 128u) ? 1 : 0;
                }
                if (cell == 'G' || cell == 'H') rw[0] = 0.0;   // (1.0, s, 0.0, true) rows: never stepped from
            } else if (e.kind == RL_ENV_CLIFF_WALKING) {
                nx[0] = w & 63u;
                rw[0] = (w & 64u) ? -100.0 : -1.0;
                tm[0] = (w & 128u) ? 1 : 0;
            } else {
                nx[0] = w & 511u;
                const uint32_t rc2 = (w >> 9) & 3u;
                rw[0] = rc2 == 0 ? -1.0 : (rc2 == 1 ? -10.0 : 20.0);
                tm[0] = (w >> 11) & 1u;
            }
            for (int i = 0; i < 3; ++i) {
                if (prob) prob[k + i] = pr[i];
                if (next) next[k + i] = nx[i];
                if (reward) reward[k + i] = rw[i];
                if (term) term[k + i] = tm[i];
            }
        }
    if (start) std::memcpy(start, e.start.data(), e.S * sizeof(double));
    return RL_OK;
}

// ---------------------------------------------------------------- Env
int rl_env_create(const rl_env_config *cfg, uint32_t n, uint64_t seed, uint64_t lane_offset, int32_t device,
                  rl_env **out) {
    if (!cfg || !out || n == 0) return fail(RL_E_ARG, "bad argument");
    *out = nullptr;
    rl_env *e = new rl_env();
    e->cfg = *cfg;
    int rc = build_env(*cfg, e->eh);
    if (rc) { delete e; return rc; }
    e->device = device;
    e->L = n;
    auto bad = [&](int code) { rl_env_destroy(e); return code; };
    if (hipSetDevice(device) != hipSuccess) return bad(fail(RL_E_HIP, "hipSetDevice failed (no GPU?)"));
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess)
        return bad(fail(RL_E_HIP, "hipStreamCreate failed"));
    if ((rc = dalloc(&e->core, n)) || (rc = dalloc(&e->rng, n)) || (rc = dalloc(&e->act_d, n)) ||
        (rc = dalloc(&e->obs_d, n)) || (rc = dalloc(&e->rew_d, n)) || (rc = dalloc(&e->term_d, n)) ||
        (rc = dalloc(&e->trans, e->eh.trans.size())) || (rc = dalloc(&e->cdf, e->eh.cdf.size())))
        return bad(rc);
    if (!e->eh.trans.empty() &&
        hipMemcpy(e->trans, e->eh.trans.data(), e->eh.trans.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bad(fail(RL_E_HIP, "table upload"));
    if (!e->eh.cdf.empty() &&
        hipMemcpy(e->cdf, e->eh.cdf.data(), e->eh.cdf.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
        return bad(fail(RL_E_HIP, "table upload"));
    KParams &p = e->kp;
    p.L = n; p.S = e->eh.S; p.A = e->eh.A; p.P = 1;
    p.core = e->core; p.rng = e->rng;
    p.trans = e->trans; p.start_cdf = e->cdf; p.n_start = (uint32_t)e->eh.cdf.size();
    p.fixed_start = e->eh.fixed_start;
    p.slippery = e->eh.slippery;
    p.max_steps = e->eh.max_steps; p.th1 = e->eh.th1; p.th2 = e->eh.th2; p.th3 = e->eh.th3;
    p.trunc_reward = e->eh.trunc_reward;
    // lane init needs aux/epi_reward: use scratch
    uint4 *aux = nullptr;
    double *er = nullptr;
    if ((rc = dalloc(&aux, n)) || (rc = dalloc(&er, n))) return bad(rc);
    p.aux = aux; p.epi_reward = er;
    launch_lane_init(cfg->kind, p, seed, lane_offset, 0.0, e->stream);
    hipError_t he = hipStreamSynchronize(e->stream);
    dfree(aux);
    dfree(er);
    p.aux = nullptr; p.epi_reward = nullptr;
    if (he != hipSuccess) return bad(fail(RL_E_HIP, hipGetErrorString(he)));
    e->ready.assign(n, 0);
    *out = e;
    return RL_OK;
}

void rl_env_destroy(rl_env *e) {
    if (!e) return;
    (void)hipSetDevice(e->device);
    if (e->view) {   // the agent owns the lanes and tables
        if (e->owner) {
            (void)hipStreamSynchronize(e->owner->stream);
            e->owner->env_view = nullptr;
        }
    } else {
        dfree(e->core); dfree(e->rng); dfree(e->trans); dfree(e->cdf);
    }
    dfree(e->act_d); dfree(e->obs_d); dfree(e->rew_d); dfree(e->term_d);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

namespace {
// the stream an Env call runs on: its own, or its agent's for a view
int env_stream(rl_env *e, hipStream_t *st) {
    if (e->view && !e->owner) return fail(RL_E_STATE, "Env view used after its agent was destroyed");
    *st = e->view ? e->owner->stream : e->stream;
    HIPC(hipSetDevice(e->device));
    return RL_OK;
}
// a view after its agent's launches: every lane's readiness from its record
// (the kernels keep LF_READY: set by a reset, cleared by a terminating step)
int view_ready_refresh(rl_env *e, hipStream_t st) {
    if (!e->view || !e->ready_stale) return RL_OK;
    std::vector<uint4> core(e->L);
    HIPC(hipMemcpyAsync(core.data(), e->kp.core, (size_t)e->L * sizeof(uint4), hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < e->L; ++i) e->ready[i] = (core[i].y & LF_READY) ? 1 : 0;
    e->ready_stale = false;
    return RL_OK;
}
}  // namespace

int rl_env_reset(rl_env *e, uint64_t *obs) {
    if (!e || !obs) return fail(RL_E_ARG, "null argument");
    hipStream_t st;
    if (int rc = env_stream(e, &st)) return rc;
    launch_env_reset(e->cfg.kind, e->kp, st, e->obs_d);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(obs, e->obs_d, e->L * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < e->L; ++i) obs[i] = rl_obs_to_reference(e->cfg.kind, (uint32_t)obs[i]);
    std::fill(e->ready.begin(), e->ready.end(), 1);
    e->ready_stale = false;
    return RL_OK;
}

int rl_env_step(rl_env *e, const uint32_t *act, uint64_t *obs, double *rew, uint8_t *term) {
    if (!e || !act || !obs || !rew || !term) return fail(RL_E_ARG, "null argument");
    hipStream_t st;
    if (int rc = env_stream(e, &st)) return rc;
    if (int rc = view_ready_refresh(e, st)) return rc;
    for (uint32_t i = 0; i < e->L; ++i) {
        if (!e->ready[i]) return fail(RL_E_NOT_READY, "EnvNotReady: lane " + std::to_string(i));
        if (act[i] >= e->eh.A) return fail(RL_E_ARG, "action out of range");
    }
    HIPC(hipMemcpyAsync(e->act_d, act, e->L * 4, hipMemcpyHostToDevice, st));
    launch_env_step(e->cfg.kind, e->kp, st, e->act_d, e->obs_d, e->rew_d, e->term_d, nullptr);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(obs, e->obs_d, e->L * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(rew, e->rew_d, e->L * 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(term, e->term_d, e->L, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < e->L; ++i) {
        obs[i] = rl_obs_to_reference(e->cfg.kind, (uint32_t)obs[i]);
        if (term[i]) e->ready[i] = 0;
    }
    return RL_OK;
}

// one lane's Env::reset / Env::step (the reference's single env): the batched
// kernels over a one-lane window of the records
int rl_env_reset_lane(rl_env *e, uint32_t lane, uint64_t *obs) {
    if (!e || !obs) return fail(RL_E_ARG, "null argument");
    if (lane >= e->L) return fail(RL_E_ARG, "lane out of range");
    hipStream_t st;
    if (int rc = env_stream(e, &st)) return rc;
    if (int rc = view_ready_refresh(e, st)) return rc;   // the other lanes' readiness
    KParams p = e->kp;
    p.L = 1; p.core += lane; p.rng += lane;
    launch_env_reset(e->cfg.kind, p, st, e->obs_d);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(obs, e->obs_d, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    *obs = rl_obs_to_reference(e->cfg.kind, (uint32_t)*obs);
    e->ready[lane] = 1;
    return RL_OK;
}

int rl_env_step_lane(rl_env *e, uint32_t lane, uint32_t action, uint64_t *obs, double *rew, uint8_t *term) {
    if (!e || !obs || !rew || !term) return fail(RL_E_ARG, "null argument");
    if (lane >= e->L) return fail(RL_E_ARG, "lane out of range");
    hipStream_t st;
    if (int rc = env_stream(e, &st)) return rc;
    if (int rc = view_ready_refresh(e, st)) return rc;
    if (!e->ready[lane]) return fail(RL_E_NOT_READY, "EnvNotReady: lane " + std::to_string(lane));
    if (action >= e->eh.A) return fail(RL_E_ARG, "action out of range");
    KParams p = e->kp;
    p.L = 1; p.core += lane; p.rng += lane;
    HIPC(hipMemcpyAsync(e->act_d, &action, 4, hipMemcpyHostToDevice, st));
    launch_env_step(e->cfg.kind, p, st, e->act_d, e->obs_d, e->rew_d, e->term_d, nullptr);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(obs, e->obs_d, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(rew, e->rew_d, 8, hipMemcpyDeviceToHost, st));
    HIPC(hipMemcpyAsync(term, e->term_d, 1, hipMemcpyDeviceToHost, st));
    HIPC(hipStreamSynchronize(st));
    *obs = rl_obs_to_reference(e->cfg.kind, (uint32_t)*obs);
    if (*term) e->ready[lane] = 0;
    return RL_OK;
}

// ---------------------------------------------------------------- Agent
int rl_agent_create(const rl_agent_config *cfg, rl_agent **out) {
    if (!cfg || !out) return fail(RL_E_ARG, "null argument");
    *out = nullptr;
    const rl_agent_config &c = *cfg;
    if (c.n_lanes == 0 || c.group_size == 0 || c.group_size > 1024 || c.sync_every == 0)
        return fail(RL_E_ARG, "need n_lanes >= 1, 1 <= group_size <= 1024, sync_every >= 1");
    if (c.agent < 0 || c.agent > 1 || c.policy < 0 || c.policy > 2 || c.selector < 0 || c.selector > 1 ||
        c.algo < 0 || c.algo > 2 || c.decay_kind < 0 || c.decay_kind > 1)
        return fail(RL_E_ARG, "enum out of range");
    if (c.policy == RL_POLICY_NEURAL) {
        if (c.group_size != 1) return fail(RL_E_ARG, "NeuralPolicy runs private agents only (group_size 1)");
        if (c.net.hidden == 0 || c.net.hidden > RL_NET_MAX_HIDDEN) return fail(RL_E_ARG, "network hidden size out of range");
        if (c.net.act_hidden < 0 || c.net.act_hidden > RL_ACT_HARD_SWISH || c.net.act_hidden == RL_ACT_SOFTMAX ||
            c.net.act_out < 0 || c.net.act_out > RL_ACT_HARD_SWISH)
            return fail(RL_E_ARG, "activation out of range (softmax: output layer only)");
    }
    rl_agent *a = new rl_agent();
    a->cfg = c;
    int rc = build_env(c.env, a->eh);
    if (rc) { delete a; return rc; }
    auto bad = [&](int code) { rl_agent_destroy(a); return code; };
    a->device = c.device;
    a->S = a->eh.S; a->A = a->eh.A; a->P = c.policy == RL_POLICY_DOUBLE ? 2 : 1;
    a->L = c.n_lanes; a->G = c.group_size; a->K = c.sync_every;
    a->priv = a->G == 1;
    if (hipSetDevice(c.device) != hipSuccess) return bad(fail(RL_E_HIP, "hipSetDevice failed (no GPU?)"));
    if (hipStreamCreateWithFlags(&a->own_stream, hipStreamNonBlocking) != hipSuccess)
        return bad(fail(RL_E_HIP, "hipStreamCreate failed"));
    a->stream = a->own_stream;
    const size_t L = a->L, SA = (size_t)a->S * a->A, PSA = a->P * SA;
    if ((rc = dalloc(&a->core, L)) || (rc = dalloc(&a->rng, L)) || (rc = dalloc(&a->aux, L)) ||
        (rc = dalloc(&a->epi_reward, L)) || (rc = dalloc(&a->stats_d, STATS_W * STATS_REP)) ||
        (rc = dalloc(&a->trans, a->eh.trans.size())) || (rc = dalloc(&a->cdf, a->eh.cdf.size())))
        return bad(rc);
    a->neural = c.policy == RL_POLICY_NEURAL;
    if (a->neural) {
        std::vector<double> feat;
        if ((rc = net_feature_table(c.env, a->eh, c.net.input, feat, a->n_in))) return bad(rc);
        a->n_params = a->n_in * c.net.hidden + c.net.hidden + c.net.hidden * a->A + a->A;
        if ((rc = dalloc(&a->net_w, (size_t)a->n_params * L)) || (rc = dalloc(&a->feat, feat.size()))) return bad(rc);
        if (hipMemcpy(a->feat, feat.data(), feat.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
            return bad(fail(RL_E_HIP, "feature upload"));
    }
    if (a->priv) {
        if (!a->neural && (rc = dalloc(&a->q_priv, PSA * L))) return bad(rc);
        // UCB counters are allocated even for eps-greedy: set_action_selector may switch
        if ((rc = dalloc(&a->n_priv, SA * L)) || (rc = dalloc(&a->t_priv, L))) return bad(rc);
    } else {
        a->delta_words = 2 * PSA + SA + 1 + 3 * PSA;
        const uint32_t n_groups = (a->L + a->G - 1) / a->G;
        a->n_groups = n_groups;
        a->merge_groups = n_groups;
        // merge buffer [PSA MAX words][delta_words SUM words]; f64 slots for every group
        if ((rc = dalloc(&a->q_base, PSA)) || (rc = dalloc(&a->n_base, SA)) || (rc = dalloc(&a->t_base, 1)) ||
            (rc = dalloc(&a->delta_own, PSA + a->delta_words)) || (rc = dalloc(&a->qslot, (size_t)n_groups * PSA)))
            return bad(rc);
        a->delta_max = a->delta_own;
        a->delta = a->delta_own + PSA;
        a->delta_cap = PSA + a->delta_words;   // the largest layout: f64 over dense rows
        if (hipMemset(a->delta_own, 0, (PSA + a->delta_words) * 8) != hipSuccess) return bad(fail(RL_E_HIP, "memset"));
        a->n_rep = std::min<uint32_t>(64u, n_groups);
        if ((rc = dalloc(&a->delta_rep, a->delta_words * a->n_rep))) return bad(rc);
        if (hipMemset(a->delta_rep, 0, a->delta_words * a->n_rep * 8) != hipSuccess)
            return bad(fail(RL_E_HIP, "memset"));
    }
    if (c.agent == RL_AGENT_TRACES) {
        if (a->S > 65535) return bad(fail(RL_E_ARG, "traces need S <= 65535"));
        // shared mode: room for the pair layout (the selector / algorithm, and so
        // the layout, may change later: agent_select_kernel)
        const bool pairs = !a->priv;
        if (pairs && SA > 32767) return bad(fail(RL_E_ARG, "shared-mode traces need S*A <= 32767"));
        const size_t SL = (pairs ? SA : (size_t)a->S) * L;   // pair lists are S*A long
        if ((rc = dalloc(&a->trace, SA * L)) || (rc = dalloc(&a->tlist, SL)) || (rc = dalloc(&a->slot_of, SL)) ||
            (rc = dalloc(&a->tcnt, L)))
            return bad(rc);
        if (hipMemset(a->trace, 0, SA * L * 8) != hipSuccess || hipMemset(a->tlist, 0, SL * 2) != hipSuccess ||
            hipMemset(a->slot_of, 0, SL * 2) != hipSuccess || hipMemset(a->tcnt, 0, (size_t)L * 4) != hipSuccess)
            return bad(fail(RL_E_HIP, "memset"));
        if (pairs) {
            a->vbits_words = (size_t)((a->S + 31) / 32) * L;
            if ((rc = dalloc(&a->vbits, a->vbits_words))) return bad(rc);
            if (hipMemset(a->vbits, 0, a->vbits_words * 4) != hipSuccess) return bad(fail(RL_E_HIP, "memset"));
        }
    }
    if (!a->eh.trans.empty() &&
        hipMemcpy(a->trans, a->eh.trans.data(), a->eh.trans.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return bad(fail(RL_E_HIP, "table upload"));
    if (!a->eh.cdf.empty() &&
        hipMemcpy(a->cdf, a->eh.cdf.data(), a->eh.cdf.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
        return bad(fail(RL_E_HIP, "table upload"));
    if (hipMemset(a->stats_d, 0, STATS_W * 8 * STATS_REP) != hipSuccess) return bad(fail(RL_E_HIP, "memset"));
    if ((rc = dalloc(&a->ctl_d, 3))) return bad(rc);
    if (hipHostMalloc((void **)&a->ctl_h, 6 * 8, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&a->ctl_ev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&a->ctl_ev[1], hipEventDisableTiming) != hipSuccess)
        return bad(fail(RL_E_HIP, "loop control buffers"));

    KParams &p = a->kp;
    p.L = a->L; p.G = a->G; p.K = a->K; p.S = a->S; p.A = a->A; p.P = a->P;
    p.core = a->core; p.rng = a->rng; p.aux = a->aux; p.epi_reward = a->epi_reward;
    p.q_base = a->q_base; p.n_base = a->n_base; p.t_base = a->t_base;
    p.delta = a->delta;
    p.delta_rep = a->delta_rep;
    p.n_rep = a->n_rep;
    p.delta_words = (uint32_t)a->delta_words;
    p.sum_words = (uint32_t)a->delta_words;
    p.q_priv = a->q_priv; p.n_priv = a->n_priv; p.t_priv = a->t_priv;
    p.net_w = a->net_w; p.feat = a->feat; p.n_in = a->n_in; p.n_hidden = c.net.hidden; p.n_params = a->n_params;
    p.act1 = c.net.act_hidden; p.act2 = c.net.act_out;
    p.trace = a->trace; p.tlist = a->tlist; p.slot_of = a->slot_of; p.tcnt = a->tcnt; p.vbits = a->vbits;
    p.trans = a->trans; p.start_cdf = a->cdf; p.n_start = (uint32_t)a->eh.cdf.size();
    p.fixed_start = a->eh.fixed_start;
    p.slippery = a->eh.slippery;
    p.max_steps = a->eh.max_steps; p.th1 = a->eh.th1; p.th2 = a->eh.th2; p.th3 = a->eh.th3;
    p.trunc_reward = a->eh.trunc_reward;
    p.target_episodes = 0; p.eval_at = 0; p.eval_div = 0; p.eval_episodes = c.eval_episodes; p.eval_only = 0;
    p.stats = a->stats_d;
    p.rec = nullptr;
    agent_sync_params(a);
    if ((rc = agent_select_kernel(a))) return bad(rc);
    launch_lane_init(c.env.kind, p, c.seed, c.lane_offset, c.eps0, a->stream);
    if (hipGetLastError() != hipSuccess) return bad(fail(RL_E_HIP, "lane init launch"));
    if ((rc = agent_reset_policy(a))) return bad(rc);
    if ((rc = agent_reset_selector(a))) return bad(rc);
    *out = a;
    return RL_OK;
}

void rl_agent_destroy(rl_agent *a) {
    if (!a) return;
    (void)hipSetDevice(a->device);
    if (a->own_stream) (void)hipStreamSynchronize(a->own_stream);
    for (auto &ev : a->events) { (void)hipEventDestroy(ev.first); (void)hipEventDestroy(ev.second); }
    dfree(a->core); dfree(a->rng); dfree(a->aux); dfree(a->epi_reward);
    dfree(a->q_base); dfree(a->n_base); dfree(a->t_base); dfree(a->delta_own); dfree(a->qslot);
    dfree(a->delta_rep);
    dfree(a->q_priv); dfree(a->n_priv); dfree(a->t_priv);
    dfree(a->trace); dfree(a->tlist); dfree(a->slot_of); dfree(a->tcnt); dfree(a->vbits); dfree(a->trans); dfree(a->cdf);
    dfree(a->stats_d); dfree(a->rec_d); dfree(a->elog_d); dfree(a->elog_cnt_d);
    dfree(a->mcnt); dfree(a->mrec); dfree(a->mslot);
    peer_free(a);
    dfree(a->net_w); dfree(a->feat); dfree(a->ctl_d); dfree(a->call_d);
    if (a->call_h) (void)hipHostFree(a->call_h);
    if (a->env_view) a->env_view->owner = nullptr;   // the view outlives its agent: calls fail with RL_E_STATE
    if (a->ctl_h) (void)hipHostFree(a->ctl_h);
    for (hipEvent_t e : a->ctl_ev)
        if (e) (void)hipEventDestroy(e);
    if (a->own_stream) (void)hipStreamDestroy(a->own_stream);
    delete a;
}

int rl_agent_set_future_q_value_func(rl_agent *a, int32_t algo) {
    if (!a || algo < 0 || algo > 2) return fail(RL_E_ARG, "bad algo");
    HIPC(hipSetDevice(a->device));
    a->cfg.algo = algo;
    agent_sync_params(a);
    return agent_recheck_repr(a);
}

int rl_agent_set_action_selector(rl_agent *a, int32_t sel, double eps0, double eps_decay, double eps_final,
                                 int32_t decay_kind, double ucb_c) {
    if (!a || sel < 0 || sel > 1 || decay_kind < 0 || decay_kind > 1) return fail(RL_E_ARG, "bad selector");
    HIPC(hipSetDevice(a->device));
    a->cfg.selector = sel;
    a->cfg.eps0 = eps0; a->cfg.eps_decay = eps_decay; a->cfg.eps_final = eps_final;
    a->cfg.decay_kind = decay_kind; a->cfg.ucb_c = ucb_c;
    agent_sync_params(a);
    int rc = agent_recheck_repr(a);
    if (rc) return rc;
    return agent_reset_selector(a);
}

int rl_agent_reset(rl_agent *a) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    if (a->mcnt) {   // model.reset: no entries, no slots (mslot = index + 1, 0 = absent)
        HIPC(hipMemsetAsync(a->mcnt, 0, (size_t)a->L * 4, a->stream));
        HIPC(hipMemsetAsync(a->mslot, 0, (size_t)a->S * a->A * a->L * 4, a->stream));
    }
    int rc = agent_reset_policy(a);
    if (rc) return rc;
    return agent_reset_selector(a);
}

namespace {
// every lane starts a new episode with an empty trace set: the reference clears
// E on termination (elegibility_traces_agent.rs:98-100) and train()/evaluate()
// always begin at an episode start, so a lane left mid-episode by run() must not
// carry its set into the next call
int clear_traces(rl_agent *a) {
    if (a->tcnt) HIPC(hipMemsetAsync(a->tcnt, 0, (size_t)a->L * 4, a->stream));
    if (a->vbits) HIPC(hipMemsetAsync(a->vbits, 0, a->vbits_words * 4, a->stream));
    return RL_OK;
}
// lanes back to TRAIN at an episode start after train()/evaluate() (success or
// error), so run() keeps training (rl.h: lanes train forever)
int rearm_train(rl_agent *a) {
    a->kp.target_episodes = 0;
    a->kp.eval_at = 0;
    a->kp.eval_only = 0;
    launch_arm_full(a->kp, RL_MODE_TRAIN, 0, 0, 0.0, a->stream);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(a->stream));
    return clear_traces(a);
}
}  // namespace

int rl_agent_train(rl_agent *a, uint64_t n_episodes, uint64_t eval_at, rl_stats *out) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    // Agent::train(env, 0, ..) runs no episode (src/agent.rs:80): nothing changes
    if (n_episodes == 0) return out ? rl_agent_stats(a, out) : RL_OK;
    int rc = clear_traces(a);
    if (rc) return rc;
    launch_arm_full(a->kp, RL_MODE_TRAIN, 0, 0, 0.0, a->stream);
    HIPC(hipGetLastError());
    a->kp.target_episodes = n_episodes;
    a->kp.eval_at = eval_at;
    a->kp.eval_div = eval_at ? ~0ull / eval_at + 1ull : 0ull;   // eval_hit() in rl_train_impl.h
    a->kp.eval_only = 0;
    rc = run_until_done(a, nullptr);
    const int rc2 = rearm_train(a);
    if (rc) return rc;
    if (rc2) return rc2;
    return out ? rl_agent_stats(a, out) : RL_OK;
}

int rl_agent_evaluate(rl_agent *a, uint64_t n_episodes, rl_stats *out) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    if (n_episodes == 0) return out ? rl_agent_stats(a, out) : RL_OK;
    if (n_episodes > 0xffffffffull) return fail(RL_E_ARG, "too many evaluation episodes");
    int rc = clear_traces(a);
    if (rc) return rc;
    launch_arm_full(a->kp, RL_MODE_EVAL, (uint32_t)n_episodes, 0, 0.0, a->stream);
    HIPC(hipGetLastError());
    a->kp.target_episodes = 0;
    a->kp.eval_at = 0;
    a->kp.eval_only = 1;
    rc = run_until_done(a, nullptr);
    const int rc2 = rearm_train(a);   // back to training mode (a new episode on the next call)
    if (rc) return rc;
    if (rc2) return rc2;
    return out ? rl_agent_stats(a, out) : RL_OK;
}

int rl_agent_run(rl_agent *a, uint32_t n) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    for (uint32_t i = 0; i < n; ++i) {
        const int rc = launch_and_merge(a);
        if (rc) return rc;
    }
    return RL_OK;
}

int rl_agent_synchronize(rl_agent *a) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    HIPC(hipStreamSynchronize(a->stream));
    return a->peer.on ? peer_check(a) : RL_OK;
}

int rl_agent_stats(rl_agent *a, rl_stats *out) {
    if (!a || !out) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(a->device));
    std::vector<unsigned long long> rep(STATS_W * STATS_REP);
    HIPC(hipMemcpyAsync(rep.data(), a->stats_d, rep.size() * 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    unsigned long long s[STATS_W] = {};
    for (uint32_t r = 0; r < STATS_REP; ++r)
        for (uint32_t i = 0; i < STATS_W; ++i) s[i] += rep[r * STATS_W + i];
    out->train_steps = s[0];
    out->eval_steps = s[1];
    out->train_episodes = s[2];
    out->eval_episodes = s[3];
    out->reward_sum_q16 = (int64_t)s[4];
    out->done_lanes = s[5];
    out->launches = a->launches;
    out->trace_states = s[7];
    out->q_clamp_hits = s[ACC_CLAMP];
    out->delta_saturations = s[ACC_SAT];
    return RL_OK;
}

int rl_agent_dims(rl_agent *a, uint32_t *S, uint32_t *A, uint32_t *P) {
    if (!a) return fail(RL_E_ARG, "null agent");
    if (S) *S = a->S;
    if (A) *A = a->A;
    if (P) *P = a->P;
    return RL_OK;
}

int rl_agent_lane_state(rl_agent *a, uint32_t *core, uint32_t *aux, size_t n) {
    if (!a || n < a->L) return fail(RL_E_ARG, "bad argument");
    HIPC(hipSetDevice(a->device));
    if (core) HIPC(hipMemcpyAsync(core, a->core, a->L * 16, hipMemcpyDeviceToHost, a->stream));
    if (aux) HIPC(hipMemcpyAsync(aux, a->aux, a->L * 16, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}

// ABI 7: the live eligibility-trace entries of every lane (shared pair layout: the
// pairs of the lanes' visited sets — a pool keeps its wave's count at the wave's
// first lane; row layout / private: visited states) at the call.  They persist
// across launches like the lane records: each launch reads them in and writes them
// out once (bench.py's algorithmic bytes for the traces rows)
int rl_agent_trace_items(rl_agent *a, uint64_t *items) {
    if (!a || !items) return fail(RL_E_ARG, "null argument");
    *items = 0;
    if (!a->tcnt) return RL_OK;
    HIPC(hipSetDevice(a->device));
    std::vector<uint32_t> t(a->L);
    HIPC(hipMemcpyAsync(t.data(), a->tcnt, (size_t)a->L * 4, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    for (uint32_t v : t) *items += v;
    return RL_OK;
}

int rl_agent_get_q(rl_agent *a, double *out, size_t n) {
    if (!a || !out) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(a->device));
    const size_t PSA = (size_t)a->P * a->S * a->A;
    if (a->neural) {   // Policy::get_values of every state: [n_lanes][S][A]
        if (n < PSA * a->L) return fail(RL_E_ARG, "output too small: need n_lanes*S*A");
        double *d = nullptr;
        HIPC(hipMalloc(&d, PSA * a->L * 8));
        launch_net_values(a->kp, d, a->stream);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(out, d, PSA * a->L * 8, hipMemcpyDeviceToHost, a->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(a->stream);
        (void)hipFree(d);
        HIPC(e);
        return RL_OK;
    }
    if (a->priv) {
        if (n < PSA * a->L) return fail(RL_E_ARG, "output too small: need n_lanes*P*S*A");
        // the device layout is the caller's, [L][P][S][A] (lane-major, rl_kparams.h)
        HIPC(hipMemcpyAsync(out, a->q_priv, PSA * a->L * 8, hipMemcpyDeviceToHost, a->stream));
        HIPC(hipStreamSynchronize(a->stream));
        return RL_OK;
    }
    if (n < PSA) return fail(RL_E_ARG, "output too small: need P*S*A");
    std::vector<double> v;
    std::vector<int64_t> w;
    const int rc = agent_table_values(a, v, w);
    if (rc) return rc;
    std::memcpy(out, v.data(), PSA * 8);
    return RL_OK;
}

int rl_agent_set_q(rl_agent *a, const double *in, size_t n) {
    if (!a || !in) return fail(RL_E_ARG, "null argument");
    if (a->neural) return fail(RL_E_STATE, "NeuralPolicy has no table: use rl_agent_set_weights");
    HIPC(hipSetDevice(a->device));
    const size_t PSA = (size_t)a->P * a->S * a->A;
    if (a->priv) {
        if (n < PSA * a->L) return fail(RL_E_ARG, "input too small");
        HIPC(hipMemcpy(a->q_priv, in, PSA * a->L * 8, hipMemcpyHostToDevice));   // [L][P][S][A] both sides
        return RL_OK;
    }
    if (n < PSA) return fail(RL_E_ARG, "input too small");
    return agent_store_table(a, in);
}

int rl_agent_q_repr(rl_agent *a, int32_t *repr) {
    if (!a || !repr) return fail(RL_E_ARG, "null argument");
    *repr = a->priv ? RL_QREPR_PRIVATE : a->qrepr;
    return RL_OK;
}

int rl_agent_set_q_mode(rl_agent *a, int32_t mode) {
    if (!a || (mode != RL_QMODE_AUTO && mode != RL_QMODE_F64)) return fail(RL_E_ARG, "bad q mode");
    if (a->priv) return RL_OK;
    HIPC(hipSetDevice(a->device));
    a->q_forced = mode == RL_QMODE_F64 ? 1 : 0;
    if (a->q_forced) return a->qrepr == RL_QREPR_FIXED40 ? agent_to_f64(a) : RL_OK;
    if (a->qrepr != RL_QREPR_F64) return RL_OK;
    // AUTO: back to the fixed point when the proof holds for the table as it is now
    std::vector<double> v;
    std::vector<int64_t> w;
    int rc = agent_table_values(a, v, w);
    if (rc) return rc;
    const double keep = a->q_abs0;
    if ((rc = agent_store_table(a, v.data()))) return rc;
    if (a->qrepr == RL_QREPR_F64) a->q_abs0 = keep;
    return RL_OK;
}

int rl_agent_get_q_raw(rl_agent *a, int64_t *out, size_t n) {
    if (!a || !out) return fail(RL_E_ARG, "null argument");
    if (a->priv) return fail(RL_E_STATE, "private mode (group_size 1) keeps f64 Q");
    const size_t PSA = (size_t)a->P * a->S * a->A;
    if (n < PSA) return fail(RL_E_ARG, "output too small");
    HIPC(hipSetDevice(a->device));
    HIPC(hipMemcpyAsync(out, a->q_base, PSA * 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}

int rl_agent_get_ucb(rl_agent *a, uint64_t *counts, size_t nc, uint64_t *t, size_t nt) {
    if (!a || !counts || !t) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(a->device));
    const size_t SA = (size_t)a->S * a->A;
    if (a->priv) {
        if (nc < SA * a->L || nt < a->L) return fail(RL_E_ARG, "output too small");
        HIPC(hipMemcpyAsync(counts, a->n_priv, SA * a->L * 8, hipMemcpyDeviceToHost, a->stream));   // [L][S][A]
        HIPC(hipMemcpyAsync(t, a->t_priv, a->L * 8, hipMemcpyDeviceToHost, a->stream));
        HIPC(hipStreamSynchronize(a->stream));
        return RL_OK;
    }
    if (nc < SA || nt < 1) return fail(RL_E_ARG, "output too small");
    HIPC(hipMemcpyAsync(counts, a->n_base, SA * 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipMemcpyAsync(t, a->t_base, 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}

int rl_agent_set_ucb(rl_agent *a, const uint64_t *counts, size_t nc, const uint64_t *t, size_t nt) {
    if (!a || !counts || !t) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(a->device));
    const size_t SA = (size_t)a->S * a->A;
    const size_t n_t = a->priv ? a->L : 1;
    if (nc < SA * n_t || nt < n_t) return fail(RL_E_ARG, "input too small");
    for (size_t i = 0; i < n_t; ++i)
        if (t[i] == 0) return fail(RL_E_ARG, "UCB t starts at 1 (upper_confidence_bound.rs:20)");
    if (a->priv) {
        HIPC(hipMemcpyAsync(a->n_priv, counts, SA * a->L * 8, hipMemcpyHostToDevice, a->stream));   // [L][S][A]
        HIPC(hipMemcpyAsync(a->t_priv, t, a->L * 8, hipMemcpyHostToDevice, a->stream));
    } else {
        HIPC(hipMemcpyAsync(a->n_base, counts, SA * 8, hipMemcpyHostToDevice, a->stream));
        HIPC(hipMemcpyAsync(a->t_base, t, 8, hipMemcpyHostToDevice, a->stream));
    }
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}

int rl_agent_get_epsilon(rl_agent *a, double *out, size_t n) {
    if (!a || !out || n < a->L) return fail(RL_E_ARG, "bad argument");
    HIPC(hipSetDevice(a->device));
    std::vector<uint4> x(a->L);
    HIPC(hipMemcpyAsync(x.data(), a->aux, a->L * 16, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    for (size_t i = 0; i < a->L; ++i) {
        const uint64_t b = ((uint64_t)x[i].y << 32) | x[i].x;
        std::memcpy(&out[i], &b, 8);
    }
    return RL_OK;
}

// ---------------------------------------------------------------- per-call Agent surface
namespace {
// call buffer of L entries: [r f64][td f64][s][a][s2][a2][action u32][term u8]
struct CallLayout {
    size_t r, td, s, a, s2, a2, act, term, total;
    explicit CallLayout(size_t L) {
        r = 0; td = 8 * L; s = 16 * L; a = s + 4 * L; s2 = a + 4 * L; a2 = s2 + 4 * L; act = a2 + 4 * L;
        term = act + 4 * L; total = term + L;
    }
};
// the reference observation (usize) of a lane as a dense state index
int dense_of(const rl_agent *a, uint64_t obs, uint32_t *out) {
    uint32_t d = 0;
    if (rl_obs_from_reference(a->cfg.env.kind, obs, &d) != RL_OK || d >= a->S)
        return fail(RL_E_ARG, "observation " + std::to_string(obs) + " is not a state of this env");
    *out = d;
    return RL_OK;
}
// get_action (op CALL_GET_ACTION) or update (CALL_UPDATE) on lanes [lane0, lane0 + n)
int agent_call(rl_agent *a, int op, uint32_t lane0, uint32_t n, const uint64_t *s, const uint32_t *act,
               const double *r, const uint8_t *term, const uint64_t *s2, const uint32_t *a2, uint32_t *action_out,
               double *td_out) {
    if (!a->priv) return fail(RL_E_STATE, "get_action / update are per-agent calls: private mode (group_size 1) only");
    if (n == 0) return RL_OK;
    if ((uint64_t)lane0 + n > a->L) return fail(RL_E_ARG, "lane out of range");
    HIPC(hipSetDevice(a->device));
    if (!a->call_d) {   // sized for every lane; a call stages only its n entries
        const CallLayout full(a->L);
        if (int rc = dalloc(&a->call_d, full.total)) return rc;
        HIPC(hipHostMalloc((void **)&a->call_h, full.total, hipHostMallocDefault));
    }
    const CallLayout cl(n);   // compact: a one-lane call moves a few bytes, not O(L)
    unsigned char *h = a->call_h;
    uint32_t *hs = (uint32_t *)(h + cl.s), *ha = (uint32_t *)(h + cl.a), *hs2 = (uint32_t *)(h + cl.s2),
             *ha2 = (uint32_t *)(h + cl.a2);
    for (uint32_t i = 0; i < n; ++i) {
        if (int rc = dense_of(a, s[i], &hs[i])) return rc;
        if (op == CALL_UPDATE) {
            if (int rc = dense_of(a, s2[i], &hs2[i])) return rc;
            if (act[i] >= a->A || a2[i] >= a->A) return fail(RL_E_ARG, "action out of range");
            ha[i] = act[i];
            ha2[i] = a2[i];
            ((double *)(h + cl.r))[i] = r[i];
            h[cl.term + i] = term[i] ? 1 : 0;
        }
    }
    // inputs: one copy of the used span (s .. term) plus r
    HIPC(hipMemcpyAsync(a->call_d + cl.s, h + cl.s, cl.total - cl.s, hipMemcpyHostToDevice, a->stream));
    if (op == CALL_UPDATE) HIPC(hipMemcpyAsync(a->call_d, h, 8 * (size_t)n, hipMemcpyHostToDevice, a->stream));
    agent_sync_params(a);
    KParams p = a->kp;
    p.call_op = op;
    p.call_lane0 = lane0;
    p.call_n = n;
    p.call.s = (const uint32_t *)(a->call_d + cl.s);
    p.call.a = (const uint32_t *)(a->call_d + cl.a);
    p.call.s2 = (const uint32_t *)(a->call_d + cl.s2);
    p.call.a2 = (const uint32_t *)(a->call_d + cl.a2);
    p.call.r = (const double *)(a->call_d + cl.r);
    p.call.term = a->call_d + cl.term;
    p.call.action_out = (uint32_t *)(a->call_d + cl.act);
    p.call.td_out = (double *)(a->call_d + cl.td);
    const hipError_t le = a->fn(p, dim3(1), dim3(1), 0, a->stream, nullptr);
    if (le != hipSuccess) return fail(RL_E_HIP, std::string("agent call launch: ") + hipGetErrorString(le));
    if (op == CALL_GET_ACTION)
        HIPC(hipMemcpyAsync(action_out, a->call_d + cl.act, 4 * (size_t)n, hipMemcpyDeviceToHost, a->stream));
    else
        HIPC(hipMemcpyAsync(td_out, a->call_d + cl.td, 8 * (size_t)n, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}
}  // namespace

int rl_agent_get_action(rl_agent *a, uint32_t lane, uint64_t obs, uint32_t *action) {
    if (!a || !action) return fail(RL_E_ARG, "null argument");
    return agent_call(a, CALL_GET_ACTION, lane, 1, &obs, nullptr, nullptr, nullptr, nullptr, nullptr, action,
                      nullptr);
}
int rl_agent_update(rl_agent *a, uint32_t lane, uint64_t curr_obs, uint32_t curr_action, double reward,
                    int32_t terminated, uint64_t next_obs, uint32_t next_action, double *td) {
    if (!a || !td) return fail(RL_E_ARG, "null argument");
    const uint8_t t = terminated ? 1 : 0;
    return agent_call(a, CALL_UPDATE, lane, 1, &curr_obs, &curr_action, &reward, &t, &next_obs, &next_action,
                      nullptr, td);
}
// every array holds n_lanes entries, and n_lanes must be the agent's lane count
// (the library read L entries of whatever the caller passed)
int rl_agent_get_actions(rl_agent *a, const uint64_t *obs, uint32_t *actions, uint64_t n_lanes) {
    if (!a || !obs || !actions) return fail(RL_E_ARG, "null argument");
    if (n_lanes != a->L)
        return fail(RL_E_ARG, "n_lanes " + std::to_string(n_lanes) + " != the agent's " + std::to_string(a->L) + " lanes");
    return agent_call(a, CALL_GET_ACTION, 0, a->L, obs, nullptr, nullptr, nullptr, nullptr, nullptr, actions, nullptr);
}
int rl_agent_updates(rl_agent *a, const uint64_t *curr_obs, const uint32_t *curr_action, const double *reward,
                     const uint8_t *terminated, const uint64_t *next_obs, const uint32_t *next_action, double *td,
                     uint64_t n_lanes) {
    if (!a || !curr_obs || !curr_action || !reward || !terminated || !next_obs || !next_action || !td)
        return fail(RL_E_ARG, "null argument");
    if (n_lanes != a->L)
        return fail(RL_E_ARG, "n_lanes " + std::to_string(n_lanes) + " != the agent's " + std::to_string(a->L) + " lanes");
    return agent_call(a, CALL_UPDATE, 0, a->L, curr_obs, curr_action, reward, terminated, next_obs, next_action,
                      nullptr, td);
}

int rl_agent_env(rl_agent *a, rl_env **out) {
    if (!a || !out) return fail(RL_E_ARG, "null argument");
    *out = nullptr;
    if (a->env_view) return fail(RL_E_STATE, "this agent already has an Env view (rl_env_destroy it first)");
    HIPC(hipSetDevice(a->device));
    rl_env *e = new rl_env();
    e->cfg = a->cfg.env;
    e->eh = a->eh;
    e->device = a->device;
    e->view = true;
    e->owner = a;
    e->L = a->L;
    int rc;
    if ((rc = dalloc(&e->act_d, e->L)) || (rc = dalloc(&e->obs_d, e->L)) || (rc = dalloc(&e->rew_d, e->L)) ||
        (rc = dalloc(&e->term_d, e->L))) {
        rl_env_destroy(e);
        return rc;
    }
    e->core = a->core; e->rng = a->rng; e->trans = a->trans; e->cdf = a->cdf;
    KParams &p = e->kp;
    p.L = e->L; p.S = a->S; p.A = a->A; p.P = 1;
    p.core = a->core; p.rng = a->rng;
    p.trans = a->trans; p.start_cdf = a->cdf; p.n_start = (uint32_t)a->eh.cdf.size();
    p.fixed_start = a->eh.fixed_start;
    p.slippery = a->eh.slippery;
    p.max_steps = a->eh.max_steps; p.th1 = a->eh.th1; p.th2 = a->eh.th2; p.th3 = a->eh.th3;
    p.trunc_reward = a->eh.trunc_reward;
    e->ready.assign(e->L, 0);
    a->env_view = e;
    *out = e;
    return RL_OK;
}

int rl_agent_set_recording(rl_agent *a, int32_t enable) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    if (enable && !a->rec_d) {
        int rc = dalloc(&a->rec_d, (size_t)a->K * a->L);
        if (rc) return rc;
    }
    a->recording = enable != 0;
    return RL_OK;
}

int rl_agent_take_records(rl_agent *a, rl_step_record *out, uint64_t cap, uint64_t *n_total) {
    if (!a) return fail(RL_E_ARG, "null agent");
    if (n_total) *n_total = a->rec_h.size();
    if (out) {
        const size_t n = std::min<size_t>(cap, a->rec_h.size());
        std::memcpy(out, a->rec_h.data(), n * sizeof(rl_step_record));
        a->rec_h.clear();
    }
    return RL_OK;
}

int rl_agent_set_reset_step(rl_agent *a, int32_t enable) {
    if (!a) return fail(RL_E_ARG, "null agent");
    a->kp.reset_step = enable ? 1 : 0;
    return RL_OK;
}

int rl_agent_set_planning(rl_agent *a, uint32_t planning_steps) {
    if (!a) return fail(RL_E_ARG, "null agent");
    if (planning_steps && !a->priv) return fail(RL_E_ARG, "Dyna planning needs group_size 1 (private agents)");
    HIPC(hipSetDevice(a->device));
    HIPC(hipStreamSynchronize(a->stream));
    dfree(a->mcnt); dfree(a->mrec); dfree(a->mslot);
    a->mcnt = a->mslot = nullptr;
    a->mrec = nullptr;
    a->plan = 0;
    if (planning_steps) {
        const size_t n = (size_t)a->S * a->A * a->L;
        int rc;
        if ((rc = dalloc(&a->mcnt, a->L)) || (rc = dalloc(&a->mrec, n)) || (rc = dalloc(&a->mslot, n)))
            return rc;
        HIPC(hipMemset(a->mcnt, 0, (size_t)a->L * 4));
        HIPC(hipMemset(a->mslot, 0, n * 4));
        a->plan = planning_steps;
    }
    agent_sync_params(a);
    return RL_OK;
}

int rl_agent_set_episode_log(rl_agent *a, uint32_t capacity_per_lane) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    HIPC(hipStreamSynchronize(a->stream));
    dfree(a->elog_d);
    dfree(a->elog_cnt_d);
    a->elog_d = nullptr;
    a->elog_cnt_d = nullptr;
    a->elog_cap = 0;
    if (capacity_per_lane) {
        int rc;
        if ((rc = dalloc(&a->elog_d, (size_t)capacity_per_lane * a->L)) || (rc = dalloc(&a->elog_cnt_d, a->L)))
            return rc;
        HIPC(hipMemset(a->elog_cnt_d, 0, (size_t)a->L * 4));
        a->elog_cap = capacity_per_lane;
    }
    agent_sync_params(a);
    return RL_OK;
}

int rl_agent_take_episodes(rl_agent *a, rl_episode_record *out, uint64_t cap, uint64_t *n_total,
                           uint64_t *n_lost) {
    if (!a) return fail(RL_E_ARG, "null agent");
    if (!a->elog_cap) return fail(RL_E_STATE, "episode log not enabled");
    HIPC(hipSetDevice(a->device));
    std::vector<uint32_t> cnt(a->L);
    std::vector<rl_episode_record> ring((size_t)a->elog_cap * a->L);
    HIPC(hipMemcpyAsync(cnt.data(), a->elog_cnt_d, (size_t)a->L * 4, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipMemcpyAsync(ring.data(), a->elog_d, ring.size() * sizeof(rl_episode_record), hipMemcpyDeviceToHost,
                        a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    uint64_t total = 0, lost = 0, w = 0;
    for (uint32_t l = 0; l < a->L; ++l) {
        const uint32_t c = cnt[l], keep = std::min(c, a->elog_cap);
        lost += c - keep;
        for (uint32_t i = c - keep; i < c; ++i, ++total)
            if (out && w < cap) out[w++] = ring[(size_t)(i % a->elog_cap) * a->L + l];
    }
    if (n_total) *n_total = total;
    if (n_lost) *n_lost = lost;
    if (out) {   // a NULL `out` only counts (the log is kept)
        HIPC(hipMemsetAsync(a->elog_cnt_d, 0, (size_t)a->L * 4, a->stream));
        HIPC(hipStreamSynchronize(a->stream));
    }
    return RL_OK;
}

int rl_agent_delta_words(rl_agent *a, uint64_t *n) {
    if (!a || !n) return fail(RL_E_ARG, "null argument");
    uint64_t mw = 0, sw = 0;
    if (!a->priv) merge_layout(a, &mw, &sw);
    *n = mw + sw;
    return RL_OK;
}
int rl_agent_delta_max_words(rl_agent *a, uint64_t *n) {
    if (!a || !n) return fail(RL_E_ARG, "null argument");
    uint64_t mw = 0, sw = 0;
    if (!a->priv) merge_layout(a, &mw, &sw);
    *n = mw;
    return RL_OK;
}
// the largest layout either representation needs: a caller-owned
// buffer of this size survives every representation switch (set_action_selector,
// set_future_q_value_func, set_q_mode, set_q)
int rl_agent_delta_cap_words(rl_agent *a, uint64_t *n) {
    if (!a || !n) return fail(RL_E_ARG, "null argument");
    *n = 0;
    if (a->priv) return RL_OK;
    // E at its largest over the selectors: Blackjack eps-greedy holds
    // 484 compact rows per table, UCB all S, and a selector switch keeps the buffer
    const uint64_t SA = (uint64_t)a->S * a->A, PSA = a->P * SA, ps = PSA;
    *n = std::max<uint64_t>(ps + 5 * ps + SA + 1, 2 * PSA + SA + 1);
    return RL_OK;
}

int rl_agent_set_delta_buffer(rl_agent *a, void *ptr, uint64_t n_words) {
    if (!a) return fail(RL_E_ARG, "null agent");
    if (a->priv) return fail(RL_E_STATE, "private mode has no merge");
    uint64_t mw, sw;
    merge_layout(a, &mw, &sw);
    if (ptr && n_words < mw + sw) return fail(RL_E_ARG, "delta buffer too small (rl_agent_delta_words)");
    a->delta_max = ptr ? (int64_t *)ptr : a->delta_own;
    a->delta_cap = ptr ? n_words : (uint64_t)a->P * a->S * a->A + a->delta_words;
    agent_sync_params(a);
    return RL_OK;
}

int rl_agent_set_merge_groups(rl_agent *a, uint64_t total_groups) {
    if (!a) return fail(RL_E_ARG, "null agent");
    a->merge_groups = total_groups ? total_groups : a->n_groups;
    a->merge_groups_set = true;
    return RL_OK;
}

int rl_agent_launch_train(rl_agent *a) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    return launch_train_kernel(a);
}

int rl_agent_launch_fold(rl_agent *a) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    // an external collective must declare the learner groups of every rank: the
    // f64 grid's headroom depends on it
    if (a->delta_max != a->delta_own && !a->comm && !a->merge_groups_set && a->qrepr == RL_QREPR_F64)
        return fail(RL_E_STATE, "external merge buffer: call rl_agent_set_merge_groups with the total learner "
                                "groups over every rank first");
    return launch_fold_kernel(a);
}

int rl_agent_launch_apply(rl_agent *a) {
    if (!a) return fail(RL_E_ARG, "null agent");
    HIPC(hipSetDevice(a->device));
    return launch_apply_kernel(a);
}

int rl_comm_unique_id(void *id_out) {
    if (!id_out) return fail(RL_E_ARG, "null argument");
    static_assert(sizeof(ncclUniqueId) == RL_COMM_ID_BYTES, "RCCL unique id size");
    ncclUniqueId id;
    NCCLC(ncclGetUniqueId(&id));
    memcpy(id_out, &id, sizeof id);
    return RL_OK;
}

int rl_comm_init(int32_t rank, int32_t world, const void *id_in, int32_t device, rl_comm **out) {
    if (!id_in || !out || world < 1 || rank < 0 || rank >= world) return fail(RL_E_ARG, "bad rank / world / id");
    *out = nullptr;
    HIPC(hipSetDevice(device));
    rl_comm *c = new rl_comm();
    c->rank = rank; c->world = world; c->device = device;
    ncclUniqueId id;
    memcpy(&id, id_in, sizeof id);
    const ncclResult_t r = ncclCommInitRank(&c->comm, world, id, rank);
    if (r != ncclSuccess) { delete c; return fail(RL_E_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)); }
    if (hipMalloc((void **)&c->word, 8) != hipSuccess) {
        (void)ncclCommDestroy(c->comm);
        delete c;
        return fail(RL_E_OOM, "comm word");
    }
    *out = c;
    return RL_OK;
}

void rl_comm_destroy(rl_comm *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->word) (void)hipFree(c->word);
    if (c->vals) (void)hipFree(c->vals);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int rl_comm_allreduce_f64(rl_comm *c, double *vals, uint32_t n, int32_t op) {
    if (!c || (!vals && n) || op < 0 || op > 2) return fail(RL_E_ARG, "bad argument");
    if (!c->comm) return fail(RL_E_STATE, "communicator aborted after a fatal error on this rank");
    HIPC(hipSetDevice(c->device));
    if (!c->stream) HIPC(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    if (n > c->n_vals) {
        if (c->vals) HIPC(hipFree(c->vals));
        c->vals = nullptr;
        c->n_vals = 0;
        HIPC(hipMalloc((void **)&c->vals, (size_t)n * 8));
        c->n_vals = n;
    }
    const ncclRedOp_t rop = op == 0 ? ncclSum : (op == 1 ? ncclMax : ncclMin);
    // n == 0 is a barrier: one word all-reduced, nothing copied back
    const uint32_t m = n ? n : 1;
    if (!c->vals) {
        HIPC(hipMalloc((void **)&c->vals, 8));
        c->n_vals = 1;
    }
    if (n) HIPC(hipMemcpyAsync(c->vals, vals, (size_t)n * 8, hipMemcpyHostToDevice, c->stream));
    NCCLC(ncclAllReduce(c->vals, c->vals, m, ncclFloat64, rop, c->comm, c->stream));
    if (n) HIPC(hipMemcpyAsync(vals, c->vals, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    return RL_OK;
}

int rl_comm_rank(rl_comm *c, int32_t *rank, int32_t *world) {
    if (!c || !rank || !world) return fail(RL_E_ARG, "null argument");
    *rank = c->rank;
    *world = c->world;
    return RL_OK;
}

// world > 1 over RCCL: the exchange regions' handles all-gathered over the
// communicator, every rank attached, one self-test merge; the peer path stays on
// only when every rank succeeded (a MIN all-reduce of the verdicts), else RCCL
namespace {
int comm_peer_setup(rl_agent *a) {
    rl_comm *c = a->comm;
    const int32_t W = c->world, R = c->rank;
    std::vector<char> hs((size_t)W * RL_PEER_HANDLE_BYTES, 0);
    int64_t ok = rl_agent_peer_handle(a, hs.data() + (size_t)R * RL_PEER_HANDLE_BYTES) == RL_OK ? 1 : 0;
    char *hd = nullptr;
    HIPC(hipMalloc((void **)&hd, hs.size()));
    HIPC(hipMemcpyAsync(hd, hs.data(), hs.size(), hipMemcpyHostToDevice, a->stream));
    const ncclResult_t nr = ncclAllGather(hd + (size_t)R * RL_PEER_HANDLE_BYTES, hd, RL_PEER_HANDLE_BYTES,
                                          ncclUint8, c->comm, a->stream);
    if (nr == ncclSuccess) HIPC(hipMemcpyAsync(hs.data(), hd, hs.size(), hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    (void)hipFree(hd);
    if (nr != ncclSuccess) return fail(RL_E_RCCL, std::string("peer handles all-gather: ") + ncclGetErrorString(nr));
    // every rank attaches (or fails) and then joins the agreement below
    auto agree = [&](int64_t mine, int64_t *all) -> int {
        HIPC(hipMemcpyAsync(c->word, &mine, 8, hipMemcpyHostToDevice, a->stream));
        NCCLC(ncclAllReduce(c->word, c->word, 1, ncclInt64, ncclMin, c->comm, a->stream));
        HIPC(hipMemcpyAsync(all, c->word, 8, hipMemcpyDeviceToHost, a->stream));
        HIPC(hipStreamSynchronize(a->stream));
        return RL_OK;
    };
    if (ok) ok = rl_agent_peer_attach(a, R, W, hs.data()) == RL_OK ? 1 : 0;
    int64_t all = 0;
    if (int rc = agree(ok, &all)) return rc;
    if (!all) {   // some rank could not map the regions: RCCL for every rank
        peer_detach(a);
        return RL_OK;
    }
    bool good = false;
    if (peer_selftest(a, &good) != RL_OK) good = false;
    if (int rc = agree(good ? 1 : 0, &all)) return rc;
    if (!all) peer_detach(a);   // (kept: the epoch count goes on from the self-test's two merges)
    return RL_OK;
}
}  // namespace

int rl_agent_set_comm(rl_agent *a, rl_comm *c) {
    if (!a) return fail(RL_E_ARG, "null agent");
    if (c && a->priv) return fail(RL_E_STATE, "private mode (group_size 1) has no merge to reduce");
    if (c && c->device != a->device) return fail(RL_E_ARG, "communicator and agent on different devices");
    HIPC(hipSetDevice(a->device));
    if (a->peer.on) peer_detach(a);
    a->comm = c;
    // the f64 merge grid's headroom counts the learner groups of every rank
    uint64_t total = a->n_groups;
    if (c) {
        const int rc = allreduce_u64(a, a->n_groups, &total);
        if (rc) return rc;
    }
    a->merge_groups = total;
    a->merge_groups_set = c != nullptr;
    const char *mp = getenv("RLAMD_MERGE");
    // RLAMD_PEER_WORLD1=1 (tests): the whole setup — the handles' all-gather over RCCL,
    // the agreement, the self-test — and the peer merges at world 1 too, so the box's
    // one GPU runs the path the driver's N-GPU runs take
    const bool w1 = getenv("RLAMD_PEER_WORLD1") != nullptr;
    if (c && (c->world > 1 || w1) && !(mp && !strcmp(mp, "rccl"))) return comm_peer_setup(a);
    return RL_OK;
}

int rl_agent_sync(rl_agent *a) {
    if (!a) return fail(RL_E_ARG, "null agent");
    if (a->priv) return RL_OK;
    HIPC(hipSetDevice(a->device));
    return merge_after_launch(a);
}

// ---------------------------------------------------------------- peer-read merge (ABI 7)
namespace {
// this rank's exchange region: uncached device memory (stores reach HBM, where a
// peer's reads over xGMI see them), two slots of the largest merge buffer either
// representation can need, and the epoch flag 128 B past them
int peer_alloc(rl_agent *a) {
    auto &pm = a->peer;
    if (pm.region) return RL_OK;
    uint64_t cap = 0;
    if (int rc = rl_agent_delta_cap_words(a, &cap)) return rc;
    pm.cap = std::max<uint64_t>(cap, 16);
    const size_t bytes = (2 * pm.cap + 32) * 8;
    if (hipExtMallocWithFlags((void **)&pm.region, bytes, hipDeviceMallocUncached) != hipSuccess) {
        pm.region = nullptr;
        return fail(RL_E_OOM, "peer exchange region (uncached)");
    }
    HIPC(hipMemset(pm.region, 0, bytes));
    if (hipMalloc((void **)&pm.err_d, 4) != hipSuccess) return fail(RL_E_OOM, "peer error word");
    HIPC(hipMemset(pm.err_d, 0, 4));
    int khz = 100000;   // the wall clock (s_memrealtime) rate
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, a->device);
    const char *e = getenv("RLAMD_PEER_TIMEOUT_S");
    pm.timeout_ticks = (int64_t)((e ? atof(e) : 120.0) * 1e3 * (khz > 0 ? khz : 100000));
    return RL_OK;
}
void peer_detach(rl_agent *a) {
    auto &pm = a->peer;
    if (a->stream) (void)hipStreamSynchronize(a->stream);
    for (int32_t r = 0; r < (int32_t)pm.bases.size(); ++r)
        if (r != pm.rank && pm.bases[r]) (void)hipIpcCloseMemHandle(pm.bases[r]);
    pm.bases.clear();
    if (pm.bases_d) (void)hipFree(pm.bases_d);
    pm.bases_d = nullptr;
    pm.on = false;
    pm.epoch = 0;
    if (pm.region) (void)hipMemset(pm.region, 0, (2 * pm.cap + 32) * 8);   // flags back to epoch 0
}
void peer_free(rl_agent *a) {
    peer_detach(a);
    if (a->peer.region) (void)hipFree(a->peer.region);
    if (a->peer.err_d) (void)hipFree(a->peer.err_d);
    a->peer.region = nullptr;
    a->peer.err_d = nullptr;
}
// a peer wait that timed out (a rank that never reached the merge)
int peer_check(rl_agent *a) {
    if (!a->peer.err_d) return RL_OK;
    uint32_t err = 0;
    HIPC(hipMemcpy(&err, a->peer.err_d, 4, hipMemcpyDeviceToHost));
    if (err) return fail(RL_E_STATE, "peer-read merge: a rank did not arrive within RLAMD_PEER_TIMEOUT_S");
    return RL_OK;
}
// a merge of known words over the peers (every rank: word i = (rank + 1)(i + 1)):
// the sums and the maxima must come back exact, else the peers cannot see each
// other's regions and the caller keeps RCCL
int peer_selftest(rl_agent *a, bool *ok) {
    auto &pm = a->peer;
    const int n = 16;
    std::vector<int64_t> v(2 * n), got(2 * n);
    for (int i = 0; i < n; ++i) v[i] = v[n + i] = (int64_t)(pm.rank + 1) * (i + 1);
    int64_t *d = nullptr;
    HIPC(hipMalloc((void **)&d, 2 * n * 8));
    int rc = RL_OK;
    if (hipMemcpyAsync(d, v.data(), 2 * n * 8, hipMemcpyHostToDevice, a->stream) != hipSuccess)
        rc = fail(RL_E_HIP, "peer self-test upload");
    const int64_t saved = pm.timeout_ticks;
    pm.timeout_ticks = std::min<int64_t>(saved, saved / 12 + 1);   // 10 s of the default 120
    if (!rc) rc = peer_allreduce(a, d, n, false);
    if (!rc) rc = peer_allreduce(a, d + n, n, true);
    pm.timeout_ticks = saved;
    if (!rc && hipMemcpyAsync(got.data(), d, 2 * n * 8, hipMemcpyDeviceToHost, a->stream) != hipSuccess)
        rc = fail(RL_E_HIP, "peer self-test read");
    if (!rc && hipStreamSynchronize(a->stream) != hipSuccess) rc = fail(RL_E_HIP, "peer self-test");
    (void)hipFree(d);
    if (rc) return rc;
    uint32_t err = 0;
    HIPC(hipMemcpy(&err, pm.err_d, 4, hipMemcpyDeviceToHost));
    const int64_t W = pm.world;
    *ok = err == 0;
    for (int i = 0; i < n && *ok; ++i)
        *ok = got[i] == (W * (W + 1) / 2) * (i + 1) && got[n + i] == W * (i + 1);
    return RL_OK;
}
}  // namespace

int rl_agent_peer_handle(rl_agent *a, void *handle_out) {
    if (!a || !handle_out) return fail(RL_E_ARG, "null argument");
    if (a->priv) return fail(RL_E_STATE, "private mode (group_size 1) has no merge to reduce");
    HIPC(hipSetDevice(a->device));
    if (int rc = peer_alloc(a)) return rc;
    static_assert(sizeof(hipIpcMemHandle_t) == RL_PEER_HANDLE_BYTES, "IPC handle size");
    hipIpcMemHandle_t h;
    HIPC(hipIpcGetMemHandle(&h, a->peer.region));
    memcpy(handle_out, &h, sizeof h);
    return RL_OK;
}

int rl_agent_peer_attach(rl_agent *a, int32_t rank, int32_t world, const void *handles) {
    if (!a || !handles || world < 1 || rank < 0 || rank >= world) return fail(RL_E_ARG, "bad rank / world / handles");
    if (a->priv) return fail(RL_E_STATE, "private mode (group_size 1) has no merge to reduce");
    HIPC(hipSetDevice(a->device));
    if (int rc = peer_alloc(a)) return rc;
    peer_detach(a);
    auto &pm = a->peer;
    pm.rank = rank;
    pm.world = world;
    pm.bases.assign(world, nullptr);
    const char *hb = (const char *)handles;
    for (int32_t r = 0; r < world; ++r) {
        if (r == rank) { pm.bases[r] = pm.region; continue; }
        hipIpcMemHandle_t h;
        memcpy(&h, hb + (size_t)r * RL_PEER_HANDLE_BYTES, sizeof h);
        void *p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            peer_detach(a);
            return fail(RL_E_HIP, std::string("hipIpcOpenMemHandle (rank ") + std::to_string(r) + "): " +
                                      hipGetErrorString(e));
        }
        pm.bases[r] = (int64_t *)p;
    }
    if (hipMalloc((void **)&pm.bases_d, world * sizeof(int64_t *)) != hipSuccess ||
        hipMemcpy(pm.bases_d, pm.bases.data(), world * sizeof(int64_t *), hipMemcpyHostToDevice) != hipSuccess) {
        peer_detach(a);
        return fail(RL_E_HIP, "peer table");
    }
    HIPC(hipMemset(pm.err_d, 0, 4));
    pm.epoch = 0;
    pm.on = world > 1 || getenv("RLAMD_PEER_WORLD1") != nullptr;
    return RL_OK;
}

int rl_agent_merge_path(rl_agent *a, int32_t *path) {
    if (!a || !path) return fail(RL_E_ARG, "null argument");
    *path = a->peer.on ? RL_MERGE_PEER : (a->comm ? RL_MERGE_RCCL : RL_MERGE_LOCAL);
    return RL_OK;
}

int rl_agent_set_stream(rl_agent *a, void *stream) {
    if (!a) return fail(RL_E_ARG, "null agent");
    a->stream = stream ? (hipStream_t)stream : a->own_stream;
    return RL_OK;
}

int rl_agent_occupancy(rl_agent *a, uint32_t *groups_per_cu, uint64_t *lds_bytes, uint32_t *block_threads) {
    if (!a || !groups_per_cu || !lds_bytes || !block_threads) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(a->device));
    agent_sync_params(a);   // the kernel choice depends on the Q representation (KParams::fq)
    int n = 0;
    HIPC(a->fn(a->kp, a->grid, a->block, a->smem, a->stream, &n));
    *groups_per_cu = (uint32_t)n;
    *lds_bytes = a->smem;
    *block_threads = a->block.x;
    return RL_OK;
}

int rl_agent_set_timing(rl_agent *a, int32_t enable) {
    if (!a) return fail(RL_E_ARG, "null agent");
    a->timing = enable != 0;
    return RL_OK;
}

int rl_agent_get_timing(rl_agent *a, double *total_ms, uint64_t *n) {
    if (!a || !total_ms || !n) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(a->device));
    HIPC(hipStreamSynchronize(a->stream));
    double tot = 0.0;
    for (auto &ev : a->events) {
        float ms = 0.f;
        HIPC(hipEventElapsedTime(&ms, ev.first, ev.second));
        tot += ms;
        (void)hipEventDestroy(ev.first);
        (void)hipEventDestroy(ev.second);
    }
    *n = a->events.size();
    *total_ms = tot;
    a->events.clear();
    return RL_OK;
}

// ---------------------------------------------------------------- KAT probes
int rl_kat_log(int32_t device, const double *x, double *out, uint32_t n) {
    if (!x || !out) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(device));
    double *dx = nullptr, *dy = nullptr;
    HIPC(hipMalloc(&dx, n * 8ull));
    HIPC(hipMalloc(&dy, n * 8ull));
    HIPC(hipMemcpy(dx, x, n * 8ull, hipMemcpyHostToDevice));
    launch_kat_log(dx, dy, n, nullptr);
    HIPC(hipGetLastError());
    HIPC(hipMemcpy(out, dy, n * 8ull, hipMemcpyDeviceToHost));
    (void)hipFree(dx);
    (void)hipFree(dy);
    return RL_OK;
}

int rl_kat_rng(int32_t device, uint64_t seed, uint64_t lane, uint32_t n, uint32_t *out) {
    if (!out) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(device));
    uint32_t *d = nullptr;
    HIPC(hipMalloc(&d, n * 4ull));
    launch_kat_rng(seed, lane, n, d, nullptr);
    HIPC(hipGetLastError());
    HIPC(hipMemcpy(out, d, n * 4ull, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return RL_OK;
}

int rl_kat_ucb(int32_t device, const double *q, const double *nc, const uint64_t *t, double c, double *out,
               uint32_t n) {
    if (!q || !nc || !t || !out) return fail(RL_E_ARG, "null argument");
    HIPC(hipSetDevice(device));
    double *dq = nullptr, *dn = nullptr, *dy = nullptr;
    uint64_t *dt = nullptr;
    HIPC(hipMalloc(&dq, n * 8ull));
    HIPC(hipMalloc(&dn, n * 8ull));
    HIPC(hipMalloc(&dy, n * 8ull));
    HIPC(hipMalloc(&dt, n * 8ull));
    HIPC(hipMemcpy(dq, q, n * 8ull, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(dn, nc, n * 8ull, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(dt, t, n * 8ull, hipMemcpyHostToDevice));
    launch_kat_ucb(dq, dn, dt, c, dy, n, nullptr);
    HIPC(hipGetLastError());
    HIPC(hipMemcpy(out, dy, n * 8ull, hipMemcpyDeviceToHost));
    (void)hipFree(dq); (void)hipFree(dn); (void)hipFree(dy); (void)hipFree(dt);
    return RL_OK;
}

}  // extern "C"

// ====================================================================== NeuralPolicy
extern "C" {

int rl_agent_net_dims(rl_agent *a, uint32_t *n_in, uint32_t *hidden, uint32_t *n_params) {
    if (!a || !n_in || !hidden || !n_params) return fail(RL_E_ARG, "null argument");
    if (!a->neural) return fail(RL_E_STATE, "not a NeuralPolicy agent");
    *n_in = a->n_in;
    *hidden = a->cfg.net.hidden;
    *n_params = a->n_params;
    return RL_OK;
}

int rl_agent_get_weights(rl_agent *a, double *out, size_t n) {
    if (!a || !out) return fail(RL_E_ARG, "null argument");
    if (!a->neural) return fail(RL_E_STATE, "not a NeuralPolicy agent");
    const size_t np = a->n_params, L = a->L;
    if (n < np * L) return fail(RL_E_ARG, "output too small: need n_lanes*n_params");
    HIPC(hipSetDevice(a->device));
    std::vector<double> tmp(np * L);
    HIPC(hipMemcpyAsync(tmp.data(), a->net_w, tmp.size() * 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    for (size_t k = 0; k < np; ++k)
        for (size_t l = 0; l < L; ++l) out[l * np + k] = tmp[k * L + l];
    return RL_OK;
}

// ABI 7: a window of lanes [lane0, lane0 + n_lanes) of a private-mode agent, in
// rl_agent_get_q's / rl_agent_get_weights' layouts, without the whole set's copy
// (2^20 lanes of cfg 7 hold 1.6 GB of Q): the bench's q_check and the full-size tests
int rl_agent_get_q_lanes(rl_agent *a, uint32_t lane0, uint32_t n_lanes, double *out, size_t n) {
    if (!a || !out) return fail(RL_E_ARG, "null argument");
    if (!a->priv) return fail(RL_E_STATE, "shared mode: one merged table (rl_agent_get_q)");
    if ((uint64_t)lane0 + n_lanes > a->L) return fail(RL_E_ARG, "lane window out of range");
    const size_t PSA = (size_t)a->P * a->S * a->A;
    if (n < PSA * n_lanes) return fail(RL_E_ARG, "output too small: need n_lanes*P*S*A");
    HIPC(hipSetDevice(a->device));
    if (a->neural) {   // get_values of every state, computed for every lane, the window copied
        double *d = nullptr;
        HIPC(hipMalloc(&d, PSA * a->L * 8));
        launch_net_values(a->kp, d, a->stream);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemcpyAsync(out, d + PSA * lane0, PSA * n_lanes * 8, hipMemcpyDeviceToHost, a->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(a->stream);
        (void)hipFree(d);
        HIPC(e);
        return RL_OK;
    }
    HIPC(hipMemcpyAsync(out, a->q_priv + PSA * lane0, PSA * n_lanes * 8, hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}
int rl_agent_get_weights_lanes(rl_agent *a, uint32_t lane0, uint32_t n_lanes, double *out, size_t n) {
    if (!a || !out) return fail(RL_E_ARG, "null argument");
    if (!a->neural) return fail(RL_E_STATE, "not a NeuralPolicy agent");
    if ((uint64_t)lane0 + n_lanes > a->L) return fail(RL_E_ARG, "lane window out of range");
    const size_t np = a->n_params, L = a->L;
    if (n < np * n_lanes) return fail(RL_E_ARG, "output too small: need n_lanes*n_params");
    HIPC(hipSetDevice(a->device));
    std::vector<double> tmp(np * n_lanes);   // device [param][lane]: one strided copy
    HIPC(hipMemcpy2DAsync(tmp.data(), (size_t)n_lanes * 8, a->net_w + lane0, L * 8, (size_t)n_lanes * 8, np,
                          hipMemcpyDeviceToHost, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    for (size_t k = 0; k < np; ++k)
        for (size_t l = 0; l < n_lanes; ++l) out[l * np + k] = tmp[k * n_lanes + l];
    return RL_OK;
}

int rl_agent_set_weights(rl_agent *a, const double *in, size_t n) {
    if (!a || !in) return fail(RL_E_ARG, "null argument");
    if (!a->neural) return fail(RL_E_STATE, "not a NeuralPolicy agent");
    const size_t np = a->n_params, L = a->L;
    if (n < np * L) return fail(RL_E_ARG, "input too small: need n_lanes*n_params");
    HIPC(hipSetDevice(a->device));
    std::vector<double> tmp(np * L);
    for (size_t k = 0; k < np; ++k)
        for (size_t l = 0; l < L; ++l) tmp[k * L + l] = in[l * np + k];
    HIPC(hipMemcpyAsync(a->net_w, tmp.data(), tmp.size() * 8, hipMemcpyHostToDevice, a->stream));
    HIPC(hipStreamSynchronize(a->stream));
    return RL_OK;
}

int rl_net_features(const rl_env_config *env, int32_t input, double *out, size_t n) {
    if (!env || !out) return fail(RL_E_ARG, "null argument");
    EnvHost e;
    int rc = build_env(*env, e);
    if (rc) return rc;
    std::vector<double> feat;
    uint32_t n_in = 0;
    if ((rc = net_feature_table(*env, e, input, feat, n_in))) return rc;
    if (n < feat.size()) return fail(RL_E_ARG, "output too small: need n_states*n_in");
    std::memcpy(out, feat.data(), feat.size() * 8);
    return RL_OK;
}

int rl_kat_act(int32_t device, int32_t act, const double *x, double *f, double *fp, uint32_t n) {
    if (!x || !f || !fp) return fail(RL_E_ARG, "null argument");
    if (act < 0 || act > RL_ACT_HARD_SWISH || act == RL_ACT_SOFTMAX) return fail(RL_E_ARG, "bad activation");
    HIPC(hipSetDevice(device));
    double *dx = nullptr, *df = nullptr, *dp = nullptr;
    HIPC(hipMalloc(&dx, n * 8ull + 8));
    HIPC(hipMalloc(&df, n * 8ull + 8));
    HIPC(hipMalloc(&dp, n * 8ull + 8));
    HIPC(hipMemcpy(dx, x, n * 8ull, hipMemcpyHostToDevice));
    launch_kat_act(act, dx, df, dp, n, nullptr);
    HIPC(hipGetLastError());
    HIPC(hipMemcpy(f, df, n * 8ull, hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(fp, dp, n * 8ull, hipMemcpyDeviceToHost));
    (void)hipFree(dx); (void)hipFree(df); (void)hipFree(dp);
    return RL_OK;
}

}  // extern "C"

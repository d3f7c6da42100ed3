/*
 * ref_faithful.c — CPU BASELINE / TEST INFRASTRUCTURE ONLY (never the product path).
 *
 * A C restatement of the reference's single-env training loop written to COST
 * what the Rust binary costs, not just to compute what it computes (SURVEY
 * §8(d) "ref_faithful"): the reference's data structures are kept
 *   - Q is a hash map keyed by the observation: TabularPolicy's
 *     FxHashMap<usize, [f64; A]> (src/policy/tabular_policy.rs:11); `predict` /
 *     `get_values` copy the row or the default (:27-33), `update` is
 *     entry().or_insert(default)[a] += lr*td (:35-38).  The map is a SwissTable
 *     like hashbrown's (16-byte control groups matched with SSE2, h2 = top 7 bits,
 *     triangular probing, growth at 7/8 load) hashed with fxhash 0.2.1's
 *     FxHasher64 (write_usize: h = (rotl(h,5) ^ x) * 0x517cc1b727220a95);
 *   - UCB counters are the same kind of map of [u128; A] rows with t: u128
 *     (src/action_selection/upper_confidence_bound.rs:11-12,29-63);
 *   - Agent::train pushes every TD error into a growing Vec<f64>, rewards into
 *     Vec<f64> and episode lengths into Vec<u128> (src/agent.rs:72-116), and runs
 *     evaluate(env, 100) at every episode % eval_at == 0 (:107-113);
 *   - FrozenLakeEnv::reset copies the start distribution into a Vec and
 *     categorical_sample collects a Vec<bool> (heap allocations, as
 *     src/env/frozen_lake.rs:106-113 and src/utils.rs:33-43 do); step copies the
 *     3 transitions and draws once even when not slippery (:115-134);
 *   - the RNG is ChaCha12 with a 4-block buffer, the generator behind rand 0.8.5's
 *     ThreadRng (rand_chacha 0.3), through rand's Uniform<f64> / Uniform<usize>
 *     mappings (uniform_epsilon_greed.rs:33-34,53,62).
 * Not modelled: kdam's progress bar (one counter update per episode).
 *
 * Build with -DRF_XOSHIRO to replace ChaCha12 by the oracle's per-lane
 * xoshiro128+ stream: the run is then bit-identical to
 * oracle/rlref.c's rlo_faithful loop, which tests/test_oracle_cross.py checks —
 * two restatements written separately from the reference source agreeing.
 *
 * FrozenLake only (4x4 / 8x8, slippery or not), OneStepAgent + TabularPolicy,
 * eps-greedy or UCB, SARSA / Q-learning / Expected SARSA: cfg 1 and cfg 2 of
 * SURVEY §8(d).
 *
 * usage: ref_faithful <map8x8> <slippery> <selector> <algo> <n_episodes> <eval_at>
 *                     <repeats> <threads> [dump_q]
 *   repeats: train -> evaluate(n_episodes) -> reset, as the bins' sweep does per
 *   configuration (src/bin/frozen_lake.rs:171-215); prints one JSON line.
 */
#include <emmintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define A 4

/* ---------------------------------------------------------------- RNG */
#ifdef RF_XOSHIRO
typedef struct { uint32_t s[4]; } rng_t;
static uint64_t sm64(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void rng_init(rng_t *r, uint64_t seed, uint64_t lane) {
    uint64_t x = seed + lane * 0x632BE59BD9B4E019ull, a = sm64(&x), b = sm64(&x);
    r->s[0] = (uint32_t)a; r->s[1] = (uint32_t)(a >> 32); r->s[2] = (uint32_t)b; r->s[3] = (uint32_t)(b >> 32);
    if (!(r->s[0] | r->s[1] | r->s[2] | r->s[3])) r->s[0] = 1;
}
static inline uint32_t rng_u32(rng_t *r) {
    uint32_t *s = r->s, res = s[0] + s[3], t = s[1] << 9;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t;
    s[3] = (s[3] << 11) | (s[3] >> 21);
    return res;
}
static inline uint64_t rng_u64(rng_t *r) { uint64_t lo = rng_u32(r); return lo | ((uint64_t)rng_u32(r) << 32); }
#else
typedef struct { uint32_t key[8]; uint64_t ctr; uint32_t buf[64]; int idx; } rng_t;
#define QR(a, b, c, d) \
    a += b; d ^= a; d = (d << 16) | (d >> 16); c += d; b ^= c; b = (b << 12) | (b >> 20); \
    a += b; d ^= a; d = (d << 8) | (d >> 24);  c += d; b ^= c; b = (b << 7) | (b >> 25);
static void chacha12_block(const uint32_t key[8], uint64_t ctr, uint32_t out[16]) {
    uint32_t x[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), 0, 0};
    uint32_t in[16];
    memcpy(in, x, sizeof in);
    for (int i = 0; i < 6; ++i) {            /* 12 rounds = 6 double rounds */
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}
static void rng_refill(rng_t *r) {
    for (int b = 0; b < 4; ++b) chacha12_block(r->key, r->ctr++, r->buf + 16 * b);
    r->idx = 0;
}
static void rng_init(rng_t *r, uint64_t seed, uint64_t lane) {
    for (int i = 0; i < 8; ++i) r->key[i] = (uint32_t)((seed + lane) * 0x9E3779B97F4A7C15ull >> (4 * i)) ^ (uint32_t)i;
    r->ctr = 0;
    rng_refill(r);
}
static inline uint32_t rng_u32(rng_t *r) {
    if (r->idx >= 64) rng_refill(r);
    return r->buf[r->idx++];
}
static inline uint64_t rng_u64(rng_t *r) {   /* BlockRng::next_u64: two words, lo first */
    uint64_t lo = rng_u32(r);
    return lo | ((uint64_t)rng_u32(r) << 32);
}
#endif
/* rand 0.8.5: Uniform<f64>(0..1) = ((u64 >> 12) | 1.0) - 1.0;
 * Uniform<usize>(0..n) = widening multiply with the rejection zone */
static inline double unif01(rng_t *r) {
    union { uint64_t u; double d; } b = {(rng_u64(r) >> 12) | 0x3FF0000000000000ull};
    return b.d - 1.0;
}
static inline uint32_t unif_action(rng_t *r) {
    const uint64_t range = A, zone = UINT64_MAX - (UINT64_MAX - range + 1) % range;
    for (;;) {
        unsigned __int128 m = (unsigned __int128)rng_u64(r) * range;
        if ((uint64_t)m <= zone) return (uint32_t)(m >> 64);
    }
}

/* ---------------------------------------------------------------- FxHashMap */
static inline uint64_t fxhash_usize(uint64_t x) { return x * 0x517cc1b727220a95ull; }   /* (rotl(0,5)^x)*K */
typedef struct {
    uint8_t *ctrl;     /* cap + 16 control bytes (0x80 empty, top bit clear = full with h2) */
    uint64_t *keys;
    unsigned char *vals;   /* cap * vsz */
    size_t cap, len, vsz;
} fxmap;
static void map_init(fxmap *m, size_t vsz) { memset(m, 0, sizeof *m); m->vsz = vsz; }
static void map_free(fxmap *m) { free(m->ctrl); free(m->keys); free(m->vals); map_init(m, m->vsz); }
static void map_alloc(fxmap *m, size_t cap) {
    m->cap = cap;
    m->ctrl = (uint8_t *)malloc(cap + 16);
    memset(m->ctrl, 0x80, cap + 16);
    m->keys = (uint64_t *)malloc(cap * sizeof(uint64_t));
    m->vals = (unsigned char *)malloc(cap * m->vsz);
    m->len = 0;
}
static inline void *map_get(const fxmap *m, uint64_t key) {
    if (!m->cap) return NULL;
    const uint64_t h = fxhash_usize(key);
    const __m128i h2 = _mm_set1_epi8((char)(h >> 57));
    size_t pos = h & (m->cap - 1), stride = 0;
    for (;;) {
        const __m128i g = _mm_loadu_si128((const __m128i *)(m->ctrl + pos));
        unsigned bits = (unsigned)_mm_movemask_epi8(_mm_cmpeq_epi8(g, h2));
        while (bits) {
            const size_t i = (pos + (size_t)__builtin_ctz(bits)) & (m->cap - 1);
            if (m->keys[i] == key) return m->vals + i * m->vsz;
            bits &= bits - 1;
        }
        if (_mm_movemask_epi8(_mm_cmpeq_epi8(g, _mm_set1_epi8((char)0x80)))) return NULL;
        stride += 16;
        pos = (pos + stride) & (m->cap - 1);
    }
}
static void *map_insert_new(fxmap *m, uint64_t key);
static void map_grow(fxmap *m) {
    fxmap o = *m;
    map_alloc(m, o.cap ? o.cap * 2 : 16);
    for (size_t i = 0; i < o.cap; ++i)
        if (!(o.ctrl[i] & 0x80)) memcpy(map_insert_new(m, o.keys[i]), o.vals + i * o.vsz, o.vsz);
    free(o.ctrl); free(o.keys); free(o.vals);
}
static void *map_insert_new(fxmap *m, uint64_t key) {
    if (!m->cap || (m->len + 1) * 8 > m->cap * 7) map_grow(m);
    const uint64_t h = fxhash_usize(key);
    size_t pos = h & (m->cap - 1), stride = 0;
    for (;;) {
        const __m128i g = _mm_loadu_si128((const __m128i *)(m->ctrl + pos));
        const unsigned e = (unsigned)_mm_movemask_epi8(g);   /* top bit set = empty */
        if (e) {
            const size_t i = (pos + (size_t)__builtin_ctz(e)) & (m->cap - 1);
            m->ctrl[i] = (uint8_t)(h >> 57);
            if (i < 16) m->ctrl[m->cap + i] = m->ctrl[i];   /* mirrored tail group */
            m->keys[i] = key;
            m->len++;
            return m->vals + i * m->vsz;
        }
        stride += 16;
        pos = (pos + stride) & (m->cap - 1);
    }
}
/* entry(key).or_insert(dflt) */
static inline void *map_entry(fxmap *m, uint64_t key, const void *dflt) {
    void *v = map_get(m, key);
    if (v) return v;
    v = map_insert_new(m, key);
    memcpy(v, dflt, m->vsz);
    return v;
}

/* ---------------------------------------------------------------- growing Vecs */
typedef struct { void *p; size_t len, cap, esz; } vec;
static inline void vec_push(vec *v, const void *x) {
    if (v->len == v->cap) {
        v->cap = v->cap ? 2 * v->cap : 4;
        v->p = realloc(v->p, v->cap * v->esz);
    }
    memcpy((char *)v->p + v->len * v->esz, x, v->esz);
    v->len++;
}
static void vec_clear(vec *v) { free(v->p); v->p = NULL; v->len = v->cap = 0; }

/* ---------------------------------------------------------------- FrozenLakeEnv */
typedef struct { double p; uint64_t s; double r; int t; } transition;   /* (f64, usize, f64, bool) */
typedef struct {
    int ready;
    uint64_t ns, pos, max_steps, curr_step;
    double *start;           /* initial_state_distrib */
    transition (*probs)[A][3];
} env_t;
static const char *MAP4[] = {"SFFF", "FHFH", "FFFH", "HFFG"};                              /* frozen_lake.rs:23 */
static const char *MAP8[] = {"SFFFFFFF", "FFFFFFFF", "FFFHFFFF", "FFFFFHFF", "FFFHFFFF", "FHHFFFHF",
                             "FHFFHFHF", "FFFHFFFG"};                                          /* :25-28 */
static void inc(int n, int row, int col, int a, int *nr, int *nc) {                         /* utils.rs:53-76 */
    *nr = row; *nc = col;
    if (a == 0) *nc = col ? col - 1 : 0;
    else if (a == 1) *nr = row + 1 < n ? row + 1 : n - 1;
    else if (a == 2) *nc = col + 1 < n ? col + 1 : n - 1;
    else if (a == 3) *nr = row ? row - 1 : 0;
}
static void env_new(env_t *e, int map8, int slippery, uint64_t max_steps) {                /* :48-102 */
    const char **map = map8 ? MAP8 : MAP4;
    const int n = map8 ? 8 : 4;
    e->ns = (uint64_t)n * n;
    e->start = (double *)calloc(e->ns, sizeof(double));
    e->probs = calloc(e->ns, sizeof *e->probs);
    int cnt = 0;
    for (uint64_t i = 0; i < e->ns; ++i) cnt += map[i / n][i % n] == 'S';
    for (uint64_t i = 0; i < e->ns; ++i)
        if (map[i / n][i % n] == 'S') e->start[i] = 1.0 / cnt;
    for (int row = 0; row < n; ++row)
        for (int col = 0; col < n; ++col) {
            const uint64_t s = (uint64_t)row * n + col;
            for (int a = 0; a < A; ++a) {
                transition *li = e->probs[s][a];
                const char c = map[row][col];
                if (c == 'G' || c == 'H') {
                    li[0] = (transition){1.0, s, 0.0, 1};
                } else {
                    const int bs[3] = {(a + 3) % 4, a, (a + 1) % 4};   /* (a-1)%4 wraps (release build) */
                    for (int k = 0; k < (slippery ? 3 : 1); ++k) {
                        const int b = slippery ? bs[k] : a;
                        int nr, nc;
                        inc(n, row, col, b, &nr, &nc);
                        const char l = map[nr][nc];
                        li[k] = (transition){slippery ? 1.0 / 3.0 : 1.0, (uint64_t)nr * n + nc, l == 'G' ? 1.0 : 0.0,
                                             l == 'G' || l == 'H'};
                    }
                }
            }
        }
    e->max_steps = max_steps;
    e->ready = 0;
}
static uint64_t categorical_sample(const double *p, size_t n, double u) {                  /* utils.rs:33-43 */
    char *r = (char *)malloc(n);              /* the collected Vec<bool> */
    double b = 0.0;
    for (size_t i = 0; i < n; ++i) { b += p[i]; r[i] = b > u; }
    uint64_t res = 0;
    char mx = r[0];
    for (size_t i = 0; i < n; ++i)
        if (r[i] > mx) { mx = r[i]; res = i; }
    free(r);
    return res;
}
static uint64_t env_reset(env_t *e, rng_t *g) {                                            /* :106-113 */
    const double u = unif01(g);
    double *v = (double *)malloc(e->ns * sizeof(double));   /* initial_state_distrib.to_vec() */
    memcpy(v, e->start, e->ns * sizeof(double));
    e->pos = categorical_sample(v, e->ns, u);
    free(v);
    e->ready = 1;
    e->curr_step = 0;
    return e->pos;
}
static int env_step(env_t *e, uint32_t a, rng_t *g, uint64_t *s2, double *r, int *term) {  /* :115-134 */
    if (!e->ready) return -1;
    if (e->curr_step >= e->max_steps) {
        e->ready = 0;
        *s2 = 0; *r = 0.0; *term = 1;
        return 0;
    }
    e->curr_step++;
    transition tr[3];
    memcpy(tr, e->probs[e->pos][a], sizeof tr);
    const double tp[3] = {tr[0].p, tr[1].p, tr[2].p};
    const double u = unif01(g);
    const uint64_t i = categorical_sample(tp, 3, u);
    e->pos = tr[i].s;
    if (tr[i].t) e->ready = 0;
    *s2 = tr[i].s; *r = tr[i].r; *term = tr[i].t;
    return 0;
}

/* ---------------------------------------------------------------- agent */
typedef struct { uint64_t lo, hi; } u128;
typedef struct {
    fxmap q;                 /* FxHashMap<usize, [f64; A]> */
    fxmap n;                 /* UCB: FxHashMap<usize, [u128; A]> */
    u128 t;
    double lr, gamma, eps, eps0, decay, eps_final, c;
    int ucb, algo;
    rng_t *g;
} agent_t;
static inline uint32_t argmax4(const double *v) {                                          /* utils.rs:1-11 */
    uint32_t r = 0;
    double m = v[0];
    for (uint32_t i = 0; i < A; ++i)
        if (v[i] > m) { m = v[i]; r = i; }
    return r;
}
static inline void predict(agent_t *ag, uint64_t s, double out[A]) {                      /* tabular_policy.rs:27-33 */
    static const double dflt[A] = {0.0, 0.0, 0.0, 0.0};
    const double *row = (const double *)map_get(&ag->q, s);
    memcpy(out, row ? row : dflt, sizeof(double) * A);
}
static inline double u128_f64(u128 x) { return (double)x.hi * 18446744073709551616.0 + (double)x.lo; }
static void ucb_values(agent_t *ag, u128 *cnt, const double *v, double *u) {              /* upper_confidence_bound.rs:33-37 */
    const double lnt = log(u128_f64(ag->t));
    for (int i = 0; i < A; ++i) u[i] = v[i] + ag->c * sqrt(lnt / (u128_f64(cnt[i]) + 2.2250738585072014e-308));
}
static uint32_t get_action(agent_t *ag, uint64_t s) {                                      /* one_step_agent.rs:48-51 */
    double v[A];
    predict(ag, s, v);
    if (!ag->ucb) {                                                                       /* uniform_epsilon_greed.rs:51-66 */
        if (ag->eps != 0.0 && unif01(ag->g) < ag->eps) return unif_action(ag->g);
        return argmax4(v);
    }
    static const u128 zero[A];
    u128 *cnt = (u128 *)map_entry(&ag->n, s, zero);
    double u[A];
    ucb_values(ag, cnt, v, u);
    const uint32_t a = argmax4(u);
    if (++cnt[a].lo == 0) cnt[a].hi++;
    if (++ag->t.lo == 0) ag->t.hi++;
    return a;
}
static void exploration_probs(agent_t *ag, uint64_t s, const double *v, double *p) {
    if (!ag->ucb) {                                                                       /* uniform_epsilon_greed.rs:72-76 */
        for (int i = 0; i < A; ++i) p[i] = ag->eps / (double)A;
        p[argmax4(v)] = 1.0 - ag->eps;
        return;
    }
    static const u128 zero[A];                                                            /* upper_confidence_bound.rs:48-63 */
    u128 *cnt = (u128 *)map_entry(&ag->n, s, zero);
    ucb_values(ag, cnt, v, p);
    double sum = 0.0;
    for (int i = 0; i < A; ++i) sum += p[i];
    for (int i = 0; i < A; ++i) p[i] /= sum;
}
static double update(agent_t *ag, uint64_t s, uint32_t a, double r, int term, uint64_t s2, uint32_t a2) {
    double nq[A], pr[A], cq[A], f = 0.0;                                                  /* one_step_agent.rs:53-86 */
    predict(ag, s2, nq);
    exploration_probs(ag, s2, nq, pr);
    if (ag->algo == 0) f = nq[a2];                                                        /* agent.rs:19-45 */
    else if (ag->algo == 1) { f = nq[0]; for (int i = 0; i < A; ++i) if (nq[i] > f) f = nq[i]; }
    else for (int i = 0; i < A; ++i) f += pr[i] * nq[i];
    predict(ag, s, cq);
    const double td = r + ag->gamma * f - cq[a];
    static const double dflt[A] = {0.0, 0.0, 0.0, 0.0};
    double *row = (double *)map_entry(&ag->q, s, dflt);                                  /* tabular_policy.rs:35-38 */
    row[a] += ag->lr * td;
    if (term && !ag->ucb) {                                                               /* decay_epsilon, :42-49 */
        const double nw = ag->eps - ag->decay;
        ag->eps = ag->eps_final > nw ? ag->eps : nw;
    }
    return td;
}
static void agent_reset(agent_t *ag) {
    map_free(&ag->q);
    map_free(&ag->n);
    ag->t = (u128){1, 0};
    ag->eps = ag->eps0;
}

typedef struct { vec rewards, lengths, errors; uint64_t steps; } history;
static void evaluate(agent_t *ag, env_t *e, uint64_t n, history *h) {                      /* agent.rs:120-141 */
    for (uint64_t ep = 0; ep < n; ++ep) {
        u128 cnt = {0, 0};
        double er = 0.0;
        uint32_t a = get_action(ag, env_reset(e, ag->g));
        for (;;) {
            cnt.lo++;
            uint64_t s2; double r; int term;
            env_step(e, a, ag->g, &s2, &r, &term);
            h->steps++;
            a = get_action(ag, s2);
            er += r;
            if (term) { vec_push(&h->rewards, &er); break; }
        }
        vec_push(&h->lengths, &cnt);
    }
}
static uint64_t train(agent_t *ag, env_t *e, uint64_t n, uint64_t eval_at, history *h) {  /* agent.rs:66-118 */
    uint64_t train_steps = 0;
    history ev = {{0, 0, 0, 8}, {0, 0, 0, 16}, {0, 0, 0, 8}, 0};
    for (uint64_t ep = 0; ep < n; ++ep) {
        u128 cnt = {0, 0};
        double er = 0.0;
        uint64_t s = env_reset(e, ag->g);
        uint32_t a = get_action(ag, s);
        for (;;) {
            cnt.lo++;
            uint64_t s2; double r; int term;
            env_step(e, a, ag->g, &s2, &r, &term);
            train_steps++;
            const uint32_t a2 = get_action(ag, s2);
            const double td = update(ag, s, a, r, term, s2, a2);
            vec_push(&h->errors, &td);
            s = s2; a = a2;
            er += r;
            if (term) { vec_push(&h->rewards, &er); break; }
        }
        if (eval_at && ep % eval_at == 0) {
            evaluate(ag, e, 100, &ev);
            vec_clear(&ev.rewards); vec_clear(&ev.lengths);
        }
        vec_push(&h->lengths, &cnt);
    }
    return train_steps;
}

/* ---------------------------------------------------------------- driver */
typedef struct {
    int map8, slip, ucb, algo, dump;
    uint64_t n, eval_at, repeats, lane, train_steps;
    double seconds;
} job;
static void *run_job(void *vp) {
    job *j = (job *)vp;
    env_t e;
    env_new(&e, j->map8, j->slip, 100);
    rng_t g;
    rng_init(&g, 0x5EED, j->lane);
    agent_t ag;
    memset(&ag, 0, sizeof ag);
    map_init(&ag.q, sizeof(double) * A);
    map_init(&ag.n, sizeof(u128) * A);
    ag.lr = 0.05; ag.gamma = 0.95; ag.eps0 = 1.0; ag.eps_final = 0.0; ag.c = 0.5;   /* frozen_lake.rs:35-73 */
    ag.decay = ag.eps0 / (0.5 * (double)j->n);                                           /* :84 */
    ag.ucb = j->ucb; ag.algo = j->algo; ag.g = &g;
    agent_reset(&ag);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t k = 0; k < j->repeats; ++k) {
        history h = {{0, 0, 0, 8}, {0, 0, 0, 16}, {0, 0, 0, 8}, 0};
        j->train_steps += train(&ag, &e, j->n, j->eval_at, &h);
        if (j->dump) {   /* Q of every state (row or default), f64 bits, then histories */
            for (uint64_t s = 0; s < e.ns; ++s) {
                double v[A];
                predict(&ag, s, v);
                for (int i = 0; i < A; ++i) { uint64_t b; memcpy(&b, &v[i], 8); printf("%016llx\n", (unsigned long long)b); }
            }
            double rs = 0.0, es = 0.0;
            for (size_t i = 0; i < h.rewards.len; ++i) rs += ((double *)h.rewards.p)[i];
            for (size_t i = 0; i < h.errors.len; ++i) es += ((double *)h.errors.p)[i];
            printf("episodes %zu errors %zu reward_sum %.17g error_sum %.17g eps %.17g\n", h.lengths.len,
                   h.errors.len, rs, es, ag.eps);
        }
        vec_clear(&h.rewards); vec_clear(&h.lengths); vec_clear(&h.errors);
        agent_reset(&ag);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    j->seconds = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    map_free(&ag.q); map_free(&ag.n);
    free(e.start); free(e.probs);
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 9) {
        fprintf(stderr, "usage: %s map8x8 slippery selector algo n_episodes eval_at repeats threads [dump]\n", argv[0]);
        return 2;
    }
    job base = {0};
    base.map8 = atoi(argv[1]); base.slip = atoi(argv[2]); base.ucb = atoi(argv[3]); base.algo = atoi(argv[4]);
    base.n = strtoull(argv[5], NULL, 10); base.eval_at = strtoull(argv[6], NULL, 10);
    base.repeats = strtoull(argv[7], NULL, 10);
    int threads = atoi(argv[8]);
    base.dump = argc > 9 ? atoi(argv[9]) : 0;
    if (threads < 1) threads = 1;
    job *jobs = (job *)calloc((size_t)threads, sizeof(job));
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; ++i) {
        jobs[i] = base;
        jobs[i].lane = (uint64_t)i;
        pthread_create(&tid[i], NULL, run_job, &jobs[i]);
    }
    uint64_t steps = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(tid[i], NULL);
        steps += jobs[i].train_steps;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    if (!base.dump)
        printf("{\"steps\": %llu, \"seconds\": %.6f, \"threads\": %d, \"steps_per_sec\": %.3f}\n",
               (unsigned long long)steps, sec, threads, (double)steps / sec);
    free(jobs); free(tid);
    return 0;
}

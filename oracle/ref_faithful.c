/*
 * ref_faithful.c — CPU BASELINE / TEST INFRASTRUCTURE ONLY (never the product path).
 *
 * A C restatement of the reference's single-env training loop written to COST
 * what the Rust binary costs, not just to compute what it computes (SURVEY
 * §8(d) "ref_faithful"): the reference's data structures are kept
 *   - Q is a hash map keyed by the observation: TabularPolicy's
 *     FxHashMap<usize, [f64; COUNT]> (src/policy/tabular_policy.rs:11); `predict` /
 *     `get_values` copy the row or the default (:27-33), `update` is
 *     entry().or_insert(default)[a] += lr*td (:35-38).  DoubleTabularPolicy keeps
 *     two such maps and a flag flipped after every update (double_tabular_policy.rs:
 *     31-67).  The map is a SwissTable like hashbrown's (16-byte control groups
 *     matched with SSE2, h2 = top 7 bits, triangular probing, growth at 7/8 load)
 *     hashed with fxhash 0.2.1's FxHasher64 (write_usize: h = (rotl(h,5) ^ x) *
 *     0x517cc1b727220a95);
 *   - UCB counters are the same kind of map of [u128; COUNT] rows with t: u128
 *     (src/action_selection/upper_confidence_bound.rs:11-12,29-63);
 *   - ElegibilityTracesAgent's trace is an FxHashMap<usize, [f64; COUNT]>: every
 *     update sweeps every entry of it, every action, and a terminated episode
 *     replaces it with a fresh map (src/agent/elegibility_traces_agent.rs:61-104);
 *   - Agent::train pushes every TD error into a growing Vec<f64>, rewards into
 *     Vec<f64> and episode lengths into Vec<u128> (src/agent.rs:72-116), and runs
 *     evaluate(env, 100) at every episode % eval_at == 0 (:107-113);
 *   - the envs as the reference builds them: FrozenLakeEnv::reset copies the start
 *     distribution into a Vec and categorical_sample collects a Vec<bool> (heap
 *     allocations, src/env/frozen_lake.rs:106-113, src/utils.rs:33-43), step copies
 *     the 3 transitions and draws once even when not slippery (:115-134);
 *     CliffWalkingEnv / TaxiEnv look up (usize, f64, bool) tables
 *     (cliff_walking.rs:74-89, taxi.rs:134-159; Taxi's reset samples its 500-state
 *     start distribution); BlackJackEnv keeps [u8; 16] hands summed with
 *     iter().sum() and returns fxhash ids of BlackJackObservation
 *     (blackjack.rs:25-27,104-163);
 *   - the RNG is ChaCha12 with a 4-block buffer, the generator behind rand 0.8.5's
 *     ThreadRng (rand_chacha 0.3), through rand's Uniform<f64> / Uniform<usize> /
 *     Uniform<u8> mappings (uniform_epsilon_greed.rs:33-34,53,62; blackjack.rs:54).
 * Not modelled: kdam's progress bar (one counter update per episode).
 *
 * Build with -DRF_XOSHIRO (linked with rlref.c) to replace ChaCha12 by the
 * oracle's per-lane xoshiro128+ stream (which also skips the
 * draws whose values the reference never looks at: FrozenLake's reset and
 * deterministic-map step draws, and the low word of a power-of-two action
 * draw, Blackjack's cards two per word, the eps test's low word when the high
 * word decides it) and libm's ln by the
 * oracle's fdlibm one (a last-ulp difference at some t reaches UCB + expected
 * SARSA's probabilities): the run is then bit-identical to
 * oracle/rlref.c's rlo_faithful loop, which tests/test_oracle_cross.py checks —
 * two restatements written separately from the reference source agreeing.
 *
 * Every tabular configuration of SURVEY §8(d) cfg 1-5: FrozenLake (4x4 / 8x8,
 * slippery or not), CliffWalking, Taxi, Blackjack; OneStepAgent or
 * ElegibilityTracesAgent; TabularPolicy or DoubleTabularPolicy; eps-greedy or UCB;
 * SARSA / Q-learning / Expected SARSA; the bins' default hyper-parameters
 * (src/bin/ *.rs: lr 0.05, gamma 0.95, eps 1 -> 0 over half the episodes, c 0.5,
 * lambda 0.5, max_steps 100).
 *
 * usage: ref_faithful <env> <map8x8> <slippery> <agent> <policy> <selector> <algo>
 *                     <n_episodes> <eval_at> <repeats> <threads> [dump_q]
 *   env 0 FrozenLake, 1 CliffWalking, 2 Taxi, 3 Blackjack; repeats: train ->
 *   reset, as the bins' sweep does per configuration (src/bin/frozen_lake.rs:
 *   171-215); prints one JSON line (dump_q: Q of every dense state, f64 bits).
 */
#include <emmintrin.h>
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>


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
/* the ChaCha block function (RFC 8439 §2.3) over words 12-15 as given and
 * `rounds` rounds; rand_chacha's ChaCha12 (rand 0.8.5's ThreadRng / StdRng core)
 * puts a 64-bit block counter in words 12-13 and its stream id (0) in 14-15 */
static void chacha_block(const uint32_t key[8], const uint32_t w[4], int rounds, uint32_t out[16]) {
    uint32_t x[16] = {0x61707865, 0x3320646e, 0x79622d32, 0x6b206574, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], w[0], w[1], w[2], w[3]};
    uint32_t in[16];
    memcpy(in, x, sizeof in);
    for (int i = 0; i < rounds / 2; ++i) {   /* double rounds: columns, then diagonals */
        QR(x[0], x[4], x[8], x[12]) QR(x[1], x[5], x[9], x[13]) QR(x[2], x[6], x[10], x[14]) QR(x[3], x[7], x[11], x[15])
        QR(x[0], x[5], x[10], x[15]) QR(x[1], x[6], x[11], x[12]) QR(x[2], x[7], x[8], x[13]) QR(x[3], x[4], x[9], x[14])
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}
static void chacha12_block(const uint32_t key[8], uint64_t ctr, uint32_t out[16]) {
    const uint32_t w[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0, 0};
    chacha_block(key, w, 12, out);
}
/* known answer (tests/test_oracle_kat.py): the same block function at 20 rounds
 * on RFC 8439 §2.3.2's key 00..1f, counter 1, nonce 00:00:00:09:00:00:00:4a:00:00:00:00,
 * and at 12 rounds on the same input; prints the 16 output words as hex */
static int kat_chacha(void) {
    uint32_t key[8], out[16];
    for (int i = 0; i < 8; ++i)
        key[i] = (uint32_t)(4 * i) | (uint32_t)(4 * i + 1) << 8 | (uint32_t)(4 * i + 2) << 16 | (uint32_t)(4 * i + 3) << 24;
    const uint32_t w[4] = {1u, 0x09000000u, 0x4a000000u, 0u};
    const int rounds[2] = {20, 12};
    printf("{");
    for (int r = 0; r < 2; ++r) {
        chacha_block(key, w, rounds[r], out);
        printf("%s\"chacha%d\": [", r ? ", " : "", rounds[r]);
        for (int i = 0; i < 16; ++i) printf("%s\"%08x\"", i ? ", " : "", out[i]);
        printf("]");
    }
    printf("}\n");
    return 0;
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
#ifdef RF_XOSHIRO
/* the oracle's stream: the eps test draws m's top 32 bits first, the low word
 * only when they leave it undecided (rlref.c eps_test) */
static inline int eps_test_xo(rng_t *r, double eps) {
    const uint32_t h = rng_u32(r);
    const double e32 = ldexp(eps, 32), hd = (double)h;
    if (hd + 1.0 <= e32) return 1;
    if (!(hd < e32)) return 0;
    union { uint64_t u; double d; } b = {((((uint64_t)h << 32) | rng_u32(r)) >> 12) | 0x3FF0000000000000ull};
    return b.d - 1.0 < eps;
}
#endif
static inline uint32_t unif_action(rng_t *r, uint32_t n) {
#ifdef RF_XOSHIRO
    /* the oracle's stream: a power-of-two range takes one u32's top bits (the
     * u64's low word is never looked at; rlref.c uniform_action) */
    if (n >= 2 && (n & (n - 1)) == 0) return rng_u32(r) >> (32 - __builtin_ctz(n));
#endif
    const uint64_t range = n, zone = UINT64_MAX - (UINT64_MAX - range + 1) % range;
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


#define MAXA 6
enum { ENV_FL = 0, ENV_CW = 1, ENV_TAXI = 2, ENV_BJ = 3 };

/* ---------------------------------------------------------------- envs */
typedef struct { double p; uint64_t s; double r; int t; } transition;   /* (f64, usize, f64, bool) */
typedef struct { uint64_t s; double r; int t; } outcome;                 /* (usize, f64, bool) */
typedef struct {
    int kind, ready;
    uint32_t A;
    uint64_t ns, pos, max_steps, curr_step;
    double *start;                 /* FrozenLake / Taxi initial_state_distrib */
    transition (*probs)[4][3];     /* FrozenLake */
    outcome (*obs)[MAXA];          /* CliffWalking [48][4], Taxi [500][6] */
    uint8_t player[16], dealer[16];   /* Blackjack */
    size_t pi, di;
    int pace, dace;
    int slippery;                  /* FrozenLake is_slippery */
} env_t;
static const char *MAP4[] = {"SFFF", "FHFH", "FFFH", "HFFG"};                              /* frozen_lake.rs:23 */
static const char *MAP8[] = {"SFFFFFFF", "FFFFFFFF", "FFFHFFFF", "FFFFFHFF", "FFFHFFFF", "FHHFFFHF",
                             "FHFFHFHF", "FFFHFFFG"};                                          /* :25-28 */
static void inc(int nrow, int ncol, int row, int col, int a, int *nr, int *nc) {            /* utils.rs:53-76 */
    *nr = row; *nc = col;
    if (a == 0) *nc = col ? col - 1 : 0;
    else if (a == 1) *nr = row + 1 < nrow ? row + 1 : nrow - 1;
    else if (a == 2) *nc = col + 1 < ncol ? col + 1 : ncol - 1;
    else if (a == 3) *nr = row ? row - 1 : 0;
}
typedef struct { uint32_t w, n; } cards_t;   /* RF_XOSHIRO: the env operation's word, halves left */
static uint8_t draw_card(rng_t *g, cards_t *cs) {   /* rand 0.8.5 Uniform<u8>(1..11): u32 widening, zone */
#ifdef RF_XOSHIRO
    /* the oracle's stream: the same rule on 16-bit halves, two cards per word,
     * per env operation (rlref.c cardsrc) */
    for (;;) {
        if (cs->n == 0) { cs->w = rng_u32(g); cs->n = 2; }
        const uint32_t h = cs->n == 2 ? cs->w >> 16 : cs->w & 0xFFFFu;
        cs->n--;
        const uint32_t m = h * 10u;
        if ((m & 0xFFFFu) <= 0xFFFFu - 6u) return (uint8_t)(1u + (m >> 16));
    }
#else
    (void)cs;
    const uint32_t zone = 0xFFFFFFFFu - 6u;
    for (;;) {
        const uint64_t m = (uint64_t)rng_u32(g) * 10u;
        if ((uint32_t)m <= zone) return (uint8_t)(1u + (uint32_t)(m >> 32));
    }
#endif
}
static void bj_init_hands(env_t *e, rng_t *g) {                                            /* blackjack.rs:60-69 */
    cards_t cs = {0, 0};
    e->player[0] = draw_card(g, &cs); e->player[1] = draw_card(g, &cs); e->pi = 2;
    e->dealer[0] = draw_card(g, &cs); e->dealer[1] = draw_card(g, &cs); e->di = 2;
    e->pace = e->player[0] == 1 || e->player[1] == 1;
    e->dace = e->dealer[0] == 1 || e->dealer[1] == 1;
}
static uint8_t hand_score(const uint8_t *h, int ace) {                                      /* :75-93 */
    uint8_t s = 0;
    for (int i = 0; i < 16; ++i) s = (uint8_t)(s + h[i]);
    return (ace && s + 10 <= 21) ? (uint8_t)(s + 10) : s;
}
static uint64_t bj_id(uint8_t p, uint8_t d, int ace) {   /* fxhash::hash(&BlackJackObservation) (:25-27) */
    const uint64_t K = 0x517cc1b727220a95ull, w[3] = {p, d, (uint64_t)(ace ? 1 : 0)};
    uint64_t h = 0;
    for (int i = 0; i < 3; ++i) h = (((h << 5) | (h >> 59)) ^ w[i]) * K;
    return h;
}
static void env_new(env_t *e, int kind, int map8, int slippery, uint64_t max_steps, rng_t *g) {
    memset(e, 0, sizeof *e);
    e->kind = kind;
    e->max_steps = max_steps;
    e->slippery = slippery;
    if (kind == ENV_FL) {                                                                     /* frozen_lake.rs:48-102 */
        const char **map = map8 ? MAP8 : MAP4;
        const int n = map8 ? 8 : 4;
        e->A = 4;
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
                for (int a = 0; a < 4; ++a) {
                    transition *li = e->probs[s][a];
                    const char c = map[row][col];
                    if (c == 'G' || c == 'H') {
                        li[0] = (transition){1.0, s, 0.0, 1};
                    } else {
                        const int bs[3] = {(a + 3) % 4, a, (a + 1) % 4};   /* (a-1)%4 wraps (release build) */
                        for (int k = 0; k < (slippery ? 3 : 1); ++k) {
                            const int b = slippery ? bs[k] : a;
                            int nr, nc;
                            inc(n, n, row, col, b, &nr, &nc);
                            const char l = map[nr][nc];
                            li[k] = (transition){slippery ? 1.0 / 3.0 : 1.0, (uint64_t)nr * n + nc,
                                                 l == 'G' ? 1.0 : 0.0, l == 'G' || l == 'H'};
                        }
                    }
                }
            }
    } else if (kind == ENV_CW) {                                                              /* cliff_walking.rs:22-59 */
        e->A = 4;
        e->ns = 48;
        e->obs = calloc(48, sizeof *e->obs);
        for (int row = 0; row < 4; ++row)
            for (int col = 0; col < 12; ++col)
                for (int a = 0; a < 4; ++a) {
                    int nr, nc;
                    inc(4, 12, row, col, a, &nr, &nc);
                    const uint64_t ns = (uint64_t)nr * 12 + nc;
                    const int win = ns == 47, lose = ns >= 37 && ns <= 46;
                    e->obs[row * 12 + col][a] = (outcome){ns, lose ? -100.0 : -1.0, lose || win};
                }
    } else if (kind == ENV_TAXI) {                                                            /* taxi.rs:57-131 */
        static const char *MAP[7] = {"+---------+", "|R: | : :G|", "| : | : : |", "| : : : : |",
                                     "| | : | : |", "|Y| : |B: |", "+---------+"};
        static const int LOCS[4][2] = {{0, 0}, {0, 4}, {4, 0}, {4, 3}};
        e->A = 6;
        e->ns = 500;
        e->start = (double *)calloc(500, sizeof(double));
        e->obs = calloc(500, sizeof *e->obs);
        double sum = 0.0;
        for (int row = 0; row < 5; ++row)
            for (int col = 0; col < 5; ++col)
                for (int pl = 0; pl < 5; ++pl)
                    for (int dl = 0; dl < 4; ++dl) {
                        const int st = ((row * 5 + col) * 5 + pl) * 4 + dl;
                        if (pl < 4 && pl != dl) { e->start[st] += 1.0; sum += 1.0; }
                        for (int a = 0; a < 6; ++a) {
                            int nrow = row, ncol = col, npl = pl, term = 0;
                            double r = -1.0;
                            if (a == 0) nrow = row + 1 < 4 ? row + 1 : 4;
                            else if (a == 1) nrow = row ? row - 1 : 0;
                            if (a == 2 && MAP[1 + row][2 * col + 2] == ':') ncol = col + 1 < 4 ? col + 1 : 4;
                            else if (a == 3 && MAP[1 + row][2 * col] == ':') ncol = col ? col - 1 : 0;
                            else if (a == 4) {
                                if (pl < 4 && row == LOCS[pl][0] && col == LOCS[pl][1]) npl = 4;
                                else r = -10.0;
                            } else if (a == 5) {
                                if (row == LOCS[dl][0] && col == LOCS[dl][1] && pl == 4) { npl = dl; term = 1; r = 20.0; }
                                else r = -10.0;
                            }
                            e->obs[st][a] = (outcome){(uint64_t)(((nrow * 5 + ncol) * 5 + npl) * 4 + dl), r, term};
                        }
                    }
        for (int i = 0; i < 500; ++i) e->start[i] /= sum;
    } else {                                                                                   /* blackjack.rs:46-58 */
        e->A = 2;
        e->ns = 2048;
        bj_init_hands(e, g);   /* BlackJackEnv::new deals (initialize_hands) */
    }
    e->ready = 0;
}
static void env_free(env_t *e) { free(e->start); free(e->probs); free(e->obs); }
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
static uint64_t env_reset(env_t *e, rng_t *g) {
    e->ready = 1;
    e->curr_step = 0;
    if (e->kind == ENV_FL) {                                                                  /* frozen_lake.rs:106-113 */
#ifdef RF_XOSHIRO
        const double u = 0.0;   /* the oracle's stream: the one-'S' maps' draw is never looked at */
#else
        const double u = unif01(g);
#endif
        double *v = (double *)malloc(e->ns * sizeof(double));   /* initial_state_distrib.to_vec() */
        memcpy(v, e->start, e->ns * sizeof(double));
        e->pos = categorical_sample(v, e->ns, u);
        free(v);
    } else if (e->kind == ENV_CW) {                                                           /* cliff_walking.rs:67-72 */
        e->pos = 36;
    } else if (e->kind == ENV_TAXI) {                                                         /* taxi.rs:135-142 */
        const double u = unif01(g);
        e->pos = categorical_sample(e->start, 500, u);
    } else {                                                                                   /* blackjack.rs:105-116 */
        memset(e->player, 0, 16);
        memset(e->dealer, 0, 16);
        bj_init_hands(e, g);
        e->pos = bj_id(hand_score(e->player, e->pace), e->dealer[0], e->pace);
    }
    return e->pos;
}
static int env_step(env_t *e, uint32_t a, rng_t *g, uint64_t *s2, double *r, int *term) {
    if (!e->ready) return -1;
    if (e->kind == ENV_BJ) {                                                                  /* blackjack.rs:118-163 */
        cards_t cs = {0, 0};
        if (a == 0) {
            e->player[e->pi++] = draw_card(g, &cs);
            const uint8_t p = hand_score(e->player, e->pace);
            if (p > 21) {
                e->ready = 0;
                *s2 = bj_id(p, hand_score(e->dealer, e->dace), e->pace); *r = -1.0; *term = 1;
                return 0;
            }
            *s2 = bj_id(p, e->dealer[0], e->pace); *r = 0.0; *term = 0;
            return 0;
        }
        e->ready = 0;
        uint8_t d = hand_score(e->dealer, e->dace);
        while (d < 17) {
            e->dealer[e->di++] = draw_card(g, &cs);
            d = hand_score(e->dealer, e->dace);
        }
        const uint8_t p = hand_score(e->player, e->pace);
        *s2 = bj_id(p, d, e->pace);
        *term = 1;
        *r = d > 21 ? 1.0 : (p > d ? 1.0 : (p < d ? -1.0 : 0.0));
        return 0;
    }
    if (e->curr_step >= e->max_steps) {                   /* frozen_lake.rs:119-122 etc. */
        e->ready = 0;
        *s2 = 0; *r = e->kind == ENV_CW ? -100.0 : 0.0; *term = 1;
        return 0;
    }
    e->curr_step++;
    if (e->kind == ENV_FL) {                                                                  /* frozen_lake.rs:123-134 */
        transition tr[3];
        memcpy(tr, e->probs[e->pos][a], sizeof tr);
        const double tp[3] = {tr[0].p, tr[1].p, tr[2].p};
#ifdef RF_XOSHIRO
        const double u = e->slippery ? unif01(g) : 0.0;   /* the oracle's stream: no unused draw */
#else
        const double u = unif01(g);                        /* drawn even when not slippery */
#endif
        const uint64_t i = categorical_sample(tp, 3, u);
        e->pos = tr[i].s;
        if (tr[i].t) e->ready = 0;
        *s2 = tr[i].s; *r = tr[i].r; *term = tr[i].t;
        return 0;
    }
    const outcome o = e->obs[e->pos][a];                 /* cliff_walking.rs:85-89, taxi.rs:154-159 */
    e->pos = o.s;
    if (o.t) e->ready = 0;
    *s2 = o.s; *r = o.r; *term = o.t;
    return 0;
}

/* ---------------------------------------------------------------- agent */
typedef struct { uint64_t lo, hi; } u128;
typedef struct {
    uint32_t A;
    int double_q, traces, ucb, algo;
    fxmap qa, qb;            /* FxHashMap<usize, [f64; A]>: TabularPolicy / DoubleTabularPolicy alpha, beta */
    int flag;                /* DoubleTabularPolicy::policy_flag (starts true) */
    fxmap n;                 /* UCB: FxHashMap<usize, [u128; A]> */
    u128 t;
    fxmap trace;             /* ElegibilityTracesAgent: FxHashMap<usize, [f64; A]> */
    double lr, gamma, lambda, eps, eps0, decay, eps_final, c;
    rng_t *g;
} agent_t;
static const double ZEROS[MAXA];
static inline uint32_t argmax_a(const double *v, uint32_t A) {                               /* utils.rs:1-11 */
    uint32_t r = 0;
    double m = v[0];
    for (uint32_t i = 0; i < A; ++i)
        if (v[i] > m) { m = v[i]; r = i; }
    return r;
}
static inline void row_or_default(const fxmap *m, uint64_t s, double *out, uint32_t A) {
    const double *row = (const double *)map_get(m, s);
    memcpy(out, row ? row : ZEROS, sizeof(double) * A);
}
static inline void predict(agent_t *ag, uint64_t s, double *out) {   /* tabular_policy.rs:27-29, double :31-39 */
    if (!ag->double_q) { row_or_default(&ag->qa, s, out, ag->A); return; }
    double a[MAXA], b[MAXA];
    row_or_default(&ag->qa, s, a, ag->A);
    row_or_default(&ag->qb, s, b, ag->A);
    for (uint32_t i = 0; i < ag->A; ++i) out[i] = (a[i] + b[i]) / 2.0;
}
static inline void get_values(agent_t *ag, uint64_t s, double *out) {   /* double_tabular_policy.rs:41-48 */
    row_or_default(ag->double_q && !ag->flag ? &ag->qb : &ag->qa, s, out, ag->A);
}
static inline void policy_update(agent_t *ag, uint64_t s, uint32_t a, double x) {   /* :50-58, tabular :35-38 */
    fxmap *m = ag->double_q && ag->flag ? &ag->qb : &ag->qa;
    double *row = (double *)map_entry(m, s, ZEROS);
    row[a] += ag->lr * x;
}
static inline double u128_f64(u128 x) { return (double)x.hi * 18446744073709551616.0 + (double)x.lo; }
#ifdef RF_XOSHIRO
/* the cross-check build: the oracle's fdlibm ln (rlref.c rlo_log), the one the
 * device shares, so the two restatements agree bit for bit */
double rlo_log(double x);
#define RF_LN rlo_log
#else
#define RF_LN log   /* f64::ln: the platform libm, as the Rust binary */
#endif
static void ucb_values(agent_t *ag, u128 *cnt, const double *v, double *u) {              /* upper_confidence_bound.rs:33-37 */
    const double lnt = RF_LN(u128_f64(ag->t));
    for (uint32_t i = 0; i < ag->A; ++i) u[i] = v[i] + ag->c * sqrt(lnt / (u128_f64(cnt[i]) + 2.2250738585072014e-308));
}
static const u128 CZERO[MAXA];
static uint32_t get_action(agent_t *ag, uint64_t s) {                                      /* one_step_agent.rs:48-51 */
    double v[MAXA];
    predict(ag, s, v);
    if (!ag->ucb) {                                                                       /* uniform_epsilon_greed.rs:51-66 */
#ifdef RF_XOSHIRO
        if (ag->eps != 0.0 && eps_test_xo(ag->g, ag->eps)) return unif_action(ag->g, ag->A);
#else
        if (ag->eps != 0.0 && unif01(ag->g) < ag->eps) return unif_action(ag->g, ag->A);
#endif
        return argmax_a(v, ag->A);
    }
    u128 *cnt = (u128 *)map_entry(&ag->n, s, CZERO);
    double u[MAXA];
    ucb_values(ag, cnt, v, u);
    const uint32_t a = argmax_a(u, ag->A);
    if (++cnt[a].lo == 0) cnt[a].hi++;
    if (++ag->t.lo == 0) ag->t.hi++;
    return a;
}
static void exploration_probs(agent_t *ag, uint64_t s, const double *v, double *p) {
    const uint32_t A = ag->A;
    if (!ag->ucb) {                                                                       /* uniform_epsilon_greed.rs:72-76 */
        for (uint32_t i = 0; i < A; ++i) p[i] = ag->eps / (double)A;
        p[argmax_a(v, A)] = 1.0 - ag->eps;
        return;
    }
    u128 *cnt = (u128 *)map_entry(&ag->n, s, CZERO);                                      /* upper_confidence_bound.rs:48-63 */
    ucb_values(ag, cnt, v, p);
    double sum = 0.0;
    for (uint32_t i = 0; i < A; ++i) sum += p[i];
    for (uint32_t i = 0; i < A; ++i) p[i] /= sum;
}
static double update(agent_t *ag, uint64_t s, uint32_t a, double r, int term, uint64_t s2, uint32_t a2) {
    const uint32_t A = ag->A;
    double nq[MAXA], pr[MAXA], cq[MAXA], f = 0.0;                                         /* one_step_agent.rs:53-86 */
    get_values(ag, s2, nq);
    exploration_probs(ag, s2, nq, pr);
    if (ag->algo == 0) f = nq[a2];                                                        /* agent.rs:19-45 */
    else if (ag->algo == 1) { f = nq[0]; for (uint32_t i = 0; i < A; ++i) if (nq[i] > f) f = nq[i]; }
    else for (uint32_t i = 0; i < A; ++i) f += pr[i] * nq[i];
    get_values(ag, s, cq);
    const double td = r + ag->gamma * f - cq[a];
    if (!ag->traces) {
        policy_update(ag, s, a, td);
    } else {                                                                              /* elegibility_traces_agent.rs:75-96 */
        double *ct = (double *)map_entry(&ag->trace, s, ZEROS);
        ct[a] += 1.0;
        for (size_t i = 0; i < ag->trace.cap; ++i) {     /* for (obs, trace_values) in &mut self.trace */
            if (ag->trace.ctrl[i] & 0x80) continue;
            double *tv = (double *)(ag->trace.vals + i * ag->trace.vsz);
            for (uint32_t b = 0; b < A; ++b) {
                policy_update(ag, ag->trace.keys[i], b, td * tv[b]);
                tv[b] *= ag->gamma * ag->lambda;
            }
        }
    }
    if (ag->double_q) ag->flag = !ag->flag;                                               /* after_update */
    if (term) {
        if (ag->traces) map_free(&ag->trace);                                             /* trace = FxHashMap::default() */
        if (!ag->ucb) {                                                                   /* decay_epsilon, :42-49 */
            const double nw = ag->eps - ag->decay;
            ag->eps = ag->eps_final > nw ? ag->eps : nw;
        }
    }
    return td;
}
static void agent_reset(agent_t *ag) {   /* Agent::reset: selector + policy (the double flag is kept) */
    map_free(&ag->qa);
    map_free(&ag->qb);
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
    int env, map8, slip, traces, double_q, ucb, algo, dump;
    uint64_t n, eval_at, repeats, lane, train_steps;
    double seconds;
} job;
static uint64_t dense_to_id(const job *j, uint64_t s) {   /* the oracle's dense index -> the reference's usize obs */
    if (j->env != ENV_BJ) return s;
    return bj_id((uint8_t)(s >> 6), (uint8_t)((s >> 1) & 31u), (int)(s & 1u));
}
static void *run_job(void *vp) {
    job *j = (job *)vp;
    rng_t g;
    rng_init(&g, 0x5EED, j->lane);
    env_t e;
    env_new(&e, j->env, j->map8, j->slip, 100, &g);
    agent_t ag;
    memset(&ag, 0, sizeof ag);
    ag.A = e.A;
    map_init(&ag.qa, sizeof(double) * e.A);
    map_init(&ag.qb, sizeof(double) * e.A);
    map_init(&ag.n, sizeof(u128) * e.A);
    map_init(&ag.trace, sizeof(double) * e.A);
    ag.lr = 0.05; ag.gamma = 0.95; ag.lambda = 0.5; ag.eps0 = 1.0; ag.eps_final = 0.0; ag.c = 0.5;   /* bins' defaults */
    ag.decay = ag.eps0 / (0.5 * (double)j->n);                                           /* frozen_lake.rs:84 */
    ag.ucb = j->ucb; ag.algo = j->algo; ag.traces = j->traces; ag.double_q = j->double_q; ag.g = &g;
    ag.flag = 1;
    agent_reset(&ag);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t k = 0; k < j->repeats; ++k) {
        history h = {{0, 0, 0, 8}, {0, 0, 0, 16}, {0, 0, 0, 8}, 0};
        j->train_steps += train(&ag, &e, j->n, j->eval_at, &h);
        if (j->dump) {   /* dump 1: Q of every dense state ([P][S][A], row or default), f64 bits, then
                            the histories' summary line; dump 2: the summary line only */
            for (int tb = 0; tb < (j->dump == 1 ? (j->double_q ? 2 : 1) : 0); ++tb)
                for (uint64_t s = 0; s < e.ns; ++s) {
                    double v[MAXA];
                    row_or_default(tb ? &ag.qb : &ag.qa, dense_to_id(j, s), v, e.A);
                    for (uint32_t i = 0; i < e.A; ++i) { uint64_t b; memcpy(&b, &v[i], 8); printf("%016llx\n", (unsigned long long)b); }
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
    map_free(&ag.qa); map_free(&ag.qb); map_free(&ag.n); map_free(&ag.trace);
    env_free(&e);
    return NULL;
}

int main(int argc, char **argv) {
#ifndef RF_XOSHIRO
    if (argc == 2 && strcmp(argv[1], "kat-chacha") == 0) return kat_chacha();
#endif
    if (argc < 12) {
        fprintf(stderr, "usage: %s env map8x8 slippery agent policy selector algo n_episodes eval_at repeats threads [dump 0|1|2]\n",
                argv[0]);
        return 2;
    }
    job base = {0};
    base.env = atoi(argv[1]); base.map8 = atoi(argv[2]); base.slip = atoi(argv[3]);
    base.traces = atoi(argv[4]); base.double_q = atoi(argv[5]); base.ucb = atoi(argv[6]); base.algo = atoi(argv[7]);
    base.n = strtoull(argv[8], NULL, 10); base.eval_at = strtoull(argv[9], NULL, 10);
    base.repeats = strtoull(argv[10], NULL, 10);
    int threads = atoi(argv[11]);
    base.dump = argc > 12 ? atoi(argv[12]) : 0;
    if (threads < 1) threads = 1;
    if (base.env < 0 || base.env > 3) { fprintf(stderr, "env 0..3\n"); return 2; }
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

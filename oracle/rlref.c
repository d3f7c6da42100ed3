/*
 * rlref.c — CPU ORACLE (test infrastructure only; see rlref.h header for the
 * parity status: "parity unpinned" — KAT- and table-fixture-pinned only).
 *
 * Plain C restatement of the reference hot path.  Every function cites the
 * reference file:line it restates (paths relative to /root/reference).
 * Build: -O2 -ffp-contract=off, no fast-math (NaN/inf semantics: SURVEY F7).
 */
#include "rlref.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>



#define MIN_POSITIVE 2.2250738585072014e-308 /* f64::MIN_POSITIVE */
#define QF_NAN  1u
#define QF_PINF 2u
#define QF_NINF 4u
#define MAXS 2048
#define MAXA 6

/* ======================================================================== */
/* ln(x): fdlibm e_log.c algorithm (public, Sun 1993).  The reference calls   */
/* f64::ln (src/action_selection/upper_confidence_bound.rs:36,57), i.e. the   */
/* platform libm.  The GPU needs a bit-identical ln on host and device, so the */
/* oracle and the product both evaluate this exact operation sequence.       */
/* ======================================================================== */
typedef union { double d; uint64_t u; } dbits;

double rlo_log(double x) {
    static const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                        two54 = 1.80143985094819840000e+16,
                        Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
                        Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
                        Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                        Lg7 = 1.479819860511658591e-01;
    double hfsq, f, s, z, R, w, t1, t2, dk;
    int32_t k, hx, i, j;
    uint32_t lx;
    dbits b;
    b.d = x;
    hx = (int32_t)(b.u >> 32);
    lx = (uint32_t)b.u;
    k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | lx) == 0) return -INFINITY;
        if (hx < 0) return NAN;
        k -= 54;
        x *= two54;
        b.d = x;
        hx = (int32_t)(b.u >> 32);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    i = (hx + 0x95f64) & 0x100000;
    b.d = x;
    b.u = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (b.u & 0xffffffffu);
    x = b.d;
    k += (i >> 20);
    f = x - 1.0;
    if ((0x000fffff & (2 + hx)) < 3) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            dk = (double)k;
            return dk * ln2_hi + dk * ln2_lo;
        }
        R = f * f * (0.5 - 0.33333333333333333 * f);
        if (k == 0) return f - R;
        dk = (double)k;
        return dk * ln2_hi - ((R - dk * ln2_lo) - f);
    }
    s = f / (2.0 + f);
    dk = (double)k;
    z = s * s;
    i = hx - 0x6147a;
    w = z * z;
    j = 0x6b851 - hx;
    t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

/* ======================================================================== */
/* exp / expm1 / tanh: fdlibm e_exp.c, s_expm1.c, s_tanh.c operation         */
/* sequences (public, Sun 1993).  The reference's activations call f64::exp / */
/* f64::tanh (src/network/activation.rs:15-21,55-61,80-88), i.e. the platform */
/* libm; as for ln, host and device evaluate this one sequence so the neural  */
/* policy agrees bit for bit (tests/test_oracle_kat.py bounds it against      */
/* numpy's libm to 1 ulp).                                                    */
/* ======================================================================== */
static inline uint32_t hi_word(double x) { dbits b; b.d = x; return (uint32_t)(b.u >> 32); }
static inline uint32_t lo_word(double x) { dbits b; b.d = x; return (uint32_t)b.u; }
static inline double with_hi(double x, uint32_t hi) {
    dbits b; b.d = x; b.u = ((uint64_t)hi << 32) | (b.u & 0xffffffffull); return b.d;
}
static inline double add_exponent(double y, int k) {   /* __HI(y) += k << 20 */
    return with_hi(y, (uint32_t)((int32_t)hi_word(y) + k * (1 << 20)));
}

double rlo_exp(double x) {
    const double halF[2] = {0.5, -0.5}, huge = 1.0e+300, twom1000 = 9.33263618503218878990e-302,
                 o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02,
                 ln2HI[2] = {6.93147180369123816490e-01, -6.93147180369123816490e-01},
                 ln2LO[2] = {1.90821492927058770002e-10, -1.90821492927058770002e-10},
                 invln2 = 1.44269504088896338700e+00, P1 = 1.66666666666666019037e-01,
                 P2 = -2.77777777770155933842e-03, P3 = 6.61375632143793436117e-05,
                 P4 = -1.65339022054652515390e-06, P5 = 4.13813679705723846039e-08;
    double y, hi = 0.0, lo = 0.0, c, t;
    int k = 0;
    uint32_t hx = hi_word(x);
    const int xsb = (int)((hx >> 31) & 1u);
    hx &= 0x7fffffffu;
    if (hx >= 0x40862E42u) {
        if (hx >= 0x7ff00000u) {
            if (((hx & 0xfffffu) | lo_word(x)) != 0) return x + x;
            return xsb == 0 ? x : 0.0;
        }
        if (x > o_threshold) return huge * huge;
        if (x < u_threshold) return twom1000 * twom1000;
    }
    if (hx > 0x3fd62e42u) {
        if (hx < 0x3FF0A2B2u) {
            hi = x - ln2HI[xsb]; lo = ln2LO[xsb]; k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + halF[xsb]);
            t = (double)k;
            hi = x - t * ln2HI[0];
            lo = t * ln2LO[0];
        }
        x = hi - lo;
    } else if (hx < 0x3e300000u) {
        if (huge + x > 1.0) return 1.0 + x;
    } else {
        k = 0;
    }
    t = x * x;
    c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return 1.0 - ((x * c) / (c - 2.0) - x);
    y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi);
    if (k >= -1021) return add_exponent(y, k);
    return add_exponent(y, k + 1000) * twom1000;
}

double rlo_expm1(double x) {
    const double huge = 1.0e+300, tiny = 1.0e-300, o_threshold = 7.09782712893383973096e+02,
                 ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 invln2 = 1.44269504088896338700e+00, Q1 = -3.33333333333331316428e-02,
                 Q2 = 1.58730158725481460165e-03, Q3 = -7.93650757867487942473e-05,
                 Q4 = 4.00821782732936239552e-06, Q5 = -2.01099218183624371326e-07;
    double y, hi, lo, c = 0.0, t, e, hxs, hfx, r1;
    int k;
    uint32_t hx = hi_word(x);
    const uint32_t xsb = hx & 0x80000000u;
    hx &= 0x7fffffffu;
    if (hx >= 0x4043687Au) {
        if (hx >= 0x40862E42u) {
            if (hx >= 0x7ff00000u) {
                if (((hx & 0xfffffu) | lo_word(x)) != 0) return x + x;
                return xsb == 0 ? x : -1.0;
            }
            if (x > o_threshold) return huge * huge;
        }
        if (xsb != 0) {
            if (x + tiny < 0.0) return tiny - 1.0;
        }
    }
    if (hx > 0x3fd62e42u) {
        if (hx < 0x3FF0A2B2u) {
            if (xsb == 0) { hi = x - ln2_hi; lo = ln2_lo; k = 1; }
            else { hi = x + ln2_hi; lo = -ln2_lo; k = -1; }
        } else {
            k = (int)(invln2 * x + ((xsb == 0) ? 0.5 : -0.5));
            t = (double)k;
            hi = x - t * ln2_hi;
            lo = t * ln2_lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (hx < 0x3c900000u) {
        t = huge + x;
        return x - (t - (huge + x));
    } else {
        k = 0;
    }
    hfx = 0.5 * x;
    hxs = x * hfx;
    r1 = 1.0 + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
    t = 3.0 - r1 * hfx;
    e = hxs * ((r1 - t) / (6.0 - x * t));
    if (k == 0) return x - (x * e - hxs);
    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5 * (x - e) - 0.5;
    if (k == 1) {
        if (x < -0.25) return -2.0 * (e - (x + 0.5));
        return 1.0 + 2.0 * (x - e);
    }
    if (k <= -2 || k > 56) {
        y = 1.0 - (e - x);
        y = add_exponent(y, k);
        return y - 1.0;
    }
    if (k < 20) {
        t = with_hi(0.0, 0x3ff00000u - (0x200000u >> k));   /* 1 - 2^-k */
        y = t - (e - x);
        y = add_exponent(y, k);
    } else {
        t = with_hi(0.0, (uint32_t)((0x3ff - k) << 20));     /* 2^-k */
        y = x - (e + t);
        y += 1.0;
        y = add_exponent(y, k);
    }
    return y;
}

double rlo_tanh(double x) {
    const double tiny = 1.0e-300;
    double t, z;
    const int32_t jx = (int32_t)hi_word(x);
    const int32_t ix = jx & 0x7fffffff;
    if (ix >= 0x7ff00000) {
        if (jx >= 0) return 1.0 / x + 1.0;
        return 1.0 / x - 1.0;
    }
    if (ix < 0x40360000) {
        if (ix < 0x3c800000) return x * (1.0 + x);
        if (ix >= 0x3ff00000) {
            t = rlo_expm1(2.0 * fabs(x));
            z = 1.0 - 2.0 / (t + 2.0);
        } else {
            t = rlo_expm1(-2.0 * fabs(x));
            z = -t / (t + 2.0);
        }
    } else {
        z = 1.0 - tiny;
    }
    return jx >= 0 ? z : -z;
}

/* ======================================================================== */
/* RNG: the reference draws from rand::thread_rng() (ChaCha12, entropy       */
/* seeded) at: frozen_lake.rs:108 (reset), :126 (step); taxi.rs:137 (reset);  */
/* blackjack.rs:76 (draw_card, the env's own thread_rng handle taken at :54); */
/* uniform_epsilon_greed.rs:53 (the eps test), :62 (the random action);       */
/* random_model.rs:30 (Dyna's replay index).  All sites share one             */
/* thread-local stream.  Replacement: one xoshiro128+ stream per lane,        */
/* seeded by splitmix64(seed + lane*C); next_u64 = lo word then hi word.      */
/* ======================================================================== */
typedef struct { uint32_t s[4]; } rlo_rng;

static uint64_t splitmix64(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static void rng_seed(rlo_rng *r, uint64_t seed, uint64_t lane) {
    uint64_t x = seed + lane * 0x632BE59BD9B4E019ull;
    uint64_t a = splitmix64(&x), b = splitmix64(&x);
    r->s[0] = (uint32_t)a; r->s[1] = (uint32_t)(a >> 32);
    r->s[2] = (uint32_t)b; r->s[3] = (uint32_t)(b >> 32);
    if ((r->s[0] | r->s[1] | r->s[2] | r->s[3]) == 0) r->s[0] = 1;
}
static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
/* xoshiro128+ (Blackman & Vigna): every draw site consumes the high bits of its
 * words (UniformFloat keeps bits 12..63 of next_u64, the integer mappings use the
 * widening multiply's high word), where '+' is as good as '**' at a third of
 * the output cost on the GPU. */
static inline uint32_t next_u32(rlo_rng *r) {
    uint32_t *s = r->s;
    uint32_t result = s[0] + s[3];
    uint32_t t = s[1] << 9;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl32(s[3], 11);
    return result;
}
static inline uint64_t next_u64(rlo_rng *r) {
    uint64_t lo = next_u32(r);
    uint64_t hi = next_u32(r);
    return lo | (hi << 32);
}
void rlo_rng_stream(uint64_t seed, uint64_t lane, uint32_t n, uint32_t *out) {
    rlo_rng r;
    rng_seed(&r, seed, lane);
    for (uint32_t i = 0; i < n; ++i) out[i] = next_u32(&r);
}

/* rand 0.8.5 UniformFloat<f64>::sample for Uniform::from(0.0..1.0):
 * value1_2 = from_bits((u64 >> 12) | bits(1.0)); value0_1 = value1_2 - 1.0;
 * result = value0_1 * scale(=1.0) + low(=0.0). */
double rlo_u64_to_uniform01(uint64_t bits) {
    dbits b;
    b.u = (bits >> 12) | 0x3FF0000000000000ull;
    double v = b.d - 1.0;
    return v * 1.0 + 0.0;
}
static inline double uniform01(rlo_rng *r) { return rlo_u64_to_uniform01(next_u64(r)); }

/* eps-greedy's test u < eps, u = UniformFloat(0..1) = m * 2^-52 with m the top 52
 * bits of a u64 (uniform_epsilon_greed.rs:51-54): the stream draws m's top 32 bits
 * h first; they decide unless h*2^-32 < eps < (h+1)*2^-32, and only then is the
 * word holding m's low 20 bits drawn — the same exact test (DESIGN.md §2 "draws";
 * device: rl_device.h eps_test). */
int rlo_eps_test_words(uint32_t h, uint32_t l, double eps, int *need_low) {
    const double e32 = ldexp(eps, 32), hd = (double)h;
    *need_low = 0;
    if (hd + 1.0 <= e32) return 1;
    if (!(hd < e32)) return 0;
    *need_low = 1;
    return rlo_u64_to_uniform01(((uint64_t)h << 32) | l) < eps;
}
static int eps_test(rlo_rng *r, double eps) {
    const uint32_t h = next_u32(r);
    int need;
    int lt = rlo_eps_test_words(h, 0, eps, &need);
    if (need) lt = rlo_eps_test_words(h, next_u32(r), eps, &need);
    return lt;
}
/* rand 0.8.5 UniformInt<usize>::sample (widening multiply + rejection zone),
 * for Uniform::from(0..COUNT) (uniform_epsilon_greed.rs:34,62). */
uint32_t rlo_uniform_int_u64(uint64_t v, uint64_t range, int *reject) {
    uint64_t ints_to_reject = (UINT64_MAX - range + 1) % range;
    uint64_t zone = UINT64_MAX - ints_to_reject;
    unsigned __int128 m = (unsigned __int128)v * range;
    uint64_t hi = (uint64_t)(m >> 64), lo = (uint64_t)m;
    *reject = !(lo <= zone);
    return (uint32_t)hi;
}
/* A a power of two: the zone rejects nothing and the value is the top log2(A)
 * bits of next_u64's HIGH word — the low word is never looked at — so the
 * stream draws one u32 and takes its top bits: the same uniform over 0..A
 * (DESIGN.md §2 "draws"; device: rl_device.h uniform_action). */
static uint32_t uniform_action(rlo_rng *r, uint32_t A) {
    if (A >= 2 && (A & (A - 1)) == 0) return next_u32(r) >> (32 - __builtin_ctz(A));
    for (;;) {
        int rej;
        uint32_t a = rlo_uniform_int_u64(next_u64(r), A, &rej);
        if (!rej) return a;
    }
}
/* rand 0.8.5 Rng::gen_range(0..range) for usize = UniformInt::sample_single_inclusive
 * (RandomModel::get_info, src/model/random_model.rs:29-31): the "conservative but
 * fast" zone (range << leading_zeros(range)) - 1, widening multiply, reject lo > zone. */
uint64_t rlo_gen_index_u64(uint64_t v, uint64_t range, int *reject) {
    const uint64_t zone = (range << __builtin_clzll(range)) - 1u;
    unsigned __int128 m = (unsigned __int128)v * range;
    *reject = !((uint64_t)m <= zone);
    return (uint64_t)(m >> 64);
}
static uint32_t gen_index(rlo_rng *r, uint32_t n) {
    for (;;) {
        int rej;
        uint64_t i = rlo_gen_index_u64(next_u64(r), n, &rej);
        if (!rej) return (uint32_t)i;
    }
}

/* RandomModel (src/model/random_model.rs): IndexMap<(s,a),(s',r)> in insertion
 * order; add_info keeps the FIRST transition seen for (s,a) (entry().or_insert).
 * Stored as a sparse set: slot[k] is valid iff slot[k] < cnt && key[slot[k]] == k. */
typedef struct {
    uint32_t cnt;
    uint32_t *key, *s2, *slot;
    double *r;
} model_t;
static void model_alloc(model_t *m, size_t nsa) {
    m->cnt = 0;
    m->key = (uint32_t *)calloc(nsa, 4); m->s2 = (uint32_t *)calloc(nsa, 4);
    m->slot = (uint32_t *)calloc(nsa, 4); m->r = (double *)calloc(nsa, 8);
}
static void model_free(model_t *m) { free(m->key); free(m->s2); free(m->slot); free(m->r); memset(m, 0, sizeof *m); }
static void model_add(model_t *m, uint32_t k, uint32_t s2, double r) {
    uint32_t j = m->slot[k];
    if (j < m->cnt && m->key[j] == k) return;
    j = m->cnt++;
    m->key[j] = k; m->s2[j] = s2; m->r[j] = r; m->slot[k] = j;
}

/* rand 0.8.5 UniformInt<u8> (u32 large type) for Uniform::from(1..11)
 * (the env's dist, blackjack.rs:55, sampled at :76): range 10,
 * ints_to_reject = (2^32-10)%10 = 6. */
uint32_t rlo_uniform_card_u32(uint32_t v, int *reject) {
    const uint32_t zone = 0xFFFFFFFFu - 6u;
    uint64_t m = (uint64_t)v * 10u;
    uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
    *reject = !(lo <= zone);
    return 1u + hi;
}
/* The stream's cards (DESIGN.md §2 "cards"): the same widening-multiply-and-zone
 * rule on 16-bit halves — card 1 + (h*10 >> 16), rejected when (h*10 & 0xffff) >
 * 65535 - (2^16 % 10) — an exact uniform over 1..10 as the u32 rule is, so one u32
 * supplies two cards, high half first.  Each env operation (a deal, a hit, the
 * dealer's draws after a stick) takes its cards from its own words (cardsrc): a
 * rejected half is skipped, a half left at the operation's end is discarded. */
uint32_t rlo_uniform_card_u16(uint32_t h, int *reject) {
    const uint32_t m = (h & 0xFFFFu) * 10u;
    *reject = !((m & 0xFFFFu) <= 0xFFFFu - 6u);
    return 1u + (m >> 16);
}
typedef struct { uint32_t w, n; } cardsrc;   /* the operation's current word, halves left */
static uint32_t draw_card(rlo_rng *r, cardsrc *cs) {
    for (;;) {
        if (cs->n == 0) { cs->w = next_u32(r); cs->n = 2; }
        const uint32_t h = cs->n == 2 ? cs->w >> 16 : cs->w & 0xFFFFu;
        cs->n--;
        int rej;
        uint32_t c = rlo_uniform_card_u16(h, &rej);
        if (!rej) return c;
    }
}

/* fxhash 0.2.1 FxHasher64 over #[derive(Hash)] BlackJackObservation
 * (blackjack.rs:10-27): write_u8(p), write_u8(d), write_u8(ace as u8);
 * h = (rotl(h,5) ^ byte) * 0x517cc1b727220a95, h0 = 0. */
uint64_t rlo_blackjack_obs_id(uint32_t p, uint32_t d, uint32_t ace) {
    const uint64_t K = 0x517cc1b727220a95ull;
    uint64_t h = 0;
    uint32_t w[3] = {p & 0xff, d & 0xff, ace ? 1u : 0u};
    for (int i = 0; i < 3; ++i) h = (((h << 5) | (h >> 59)) ^ (uint64_t)w[i]) * K;
    return h;
}

/* ======================================================================== */
/* utils (src/utils.rs)                                                      */
/* ======================================================================== */
/* argmax: src/utils.rs:1-11 — first maximum, strict `>` */
static inline uint32_t argmax_d(const double *v, uint32_t n) {
    double m = v[0];
    uint32_t res = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (v[i] > m) { m = v[i]; res = i; }
    return res;
}
/* max: src/utils.rs:13-21 */
static inline double max_d(const double *v, uint32_t n) {
    double m = v[0];
    for (uint32_t i = 0; i < n; ++i)
        if (v[i] > m) m = v[i];
    return m;
}
/* categorical_sample: src/utils.rs:33-43 — running sum, first b > u, else 0 */
static uint32_t categorical_sample(const double *p, uint32_t n, double u) {
    double b = 0.0;
    for (uint32_t i = 0; i < n; ++i) {
        b += p[i];
        if (b > u) return i;
    }
    return 0;
}
/* inc: src/utils.rs:53-76 — LEFT/DOWN/RIGHT/UP with clamping */
static void inc(uint32_t nrow, uint32_t ncol, uint32_t row, uint32_t col, uint32_t a,
                uint32_t *nr, uint32_t *nc) {
    *nr = row; *nc = col;
    if (a == 0) *nc = col != 0 ? col - 1 : 0;
    else if (a == 1) *nr = row + 1 < nrow - 1 ? row + 1 : nrow - 1;
    else if (a == 2) *nc = col + 1 < ncol - 1 ? col + 1 : ncol - 1;
    else if (a == 3) *nr = row != 0 ? row - 1 : 0;
}

/* ======================================================================== */
/* environments                                                              */
/* ======================================================================== */
typedef struct {
    int kind;
    uint32_t S, A, max_steps;
    /* table envs: per (s,a) 3 outcomes */
    double prob[MAXS * MAXA * 3];
    uint32_t next[MAXS * MAXA * 3];
    double rew[MAXS * MAXA * 3];
    uint8_t term[MAXS * MAXA * 3];
    double start[MAXS];
    uint32_t n_start;
    double trunc_reward;
    int trunc_stay;      /* truncation observes the current position (FrozenLakeEdited) instead of 0 */
    uint32_t nrow, ncol; /* grid envs */
    const char **map;    /* FrozenLake maps */
    int slippery;        /* FrozenLake family: is_slippery (the step's draw is used) */
    int32_t fixed_start; /* >= 0: the start distribution is one state (no reset draw) */
} envdef;

typedef struct {
    uint32_t pos, curr_step;
    int ready;
    uint32_t p_sum, d_sum, d0, p_ace, d_ace; /* blackjack */
} envstate;

static const char *FL4[4] = {"SFFF", "FHFH", "FFFH", "HFFG"};        /* frozen_lake.rs:23 */
static const char *FL8[8] = {"SFFFFFFF", "FFFFFFFF", "FFFHFFFF", "FFFFFHFF",
                             "FFFHFFFF", "FHHFFFHF", "FHFFHFHF", "FFFHFFFG"}; /* :25-28 */
static const char *TAXI_MAP[7] = {"+---------+", "|R: | : :G|", "| : | : : |", "| : : : : |",
                                  "| | : | : |", "|Y| : |B: |", "+---------+"}; /* taxi.rs:22-30 */
static const uint32_t TAXI_LOCS[4][2] = {{0, 0}, {0, 4}, {4, 0}, {4, 3}};  /* taxi.rs:31 */

static void set_outcome(envdef *E, uint32_t s, uint32_t a, int i, double p, uint32_t n, double r,
                        int t) {
    size_t k = ((size_t)s * E->A + a) * 3 + (size_t)i;
    E->prob[k] = p; E->next[k] = n; E->rew[k] = r; E->term[k] = (uint8_t)t;
}

/* FrozenLakeEnv::new: src/env/frozen_lake.rs:48-102 */
static void build_frozen_lake(envdef *E, int map8, int slippery) {
    const char **map = map8 ? FL8 : FL4;
    uint32_t n = map8 ? 8 : 4;
    E->S = n * n; E->A = 4; E->nrow = E->ncol = n; E->map = map;
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < E->S; ++i) if (map[i / n][i % n] == 'S') cnt++;
    for (uint32_t i = 0; i < E->S; ++i) E->start[i] = map[i / n][i % n] == 'S' ? 1.0 / (double)cnt : 0.0;
    E->n_start = E->S;
    for (uint32_t row = 0; row < n; ++row)
        for (uint32_t col = 0; col < n; ++col) {
            uint32_t s = row * n + col;
            for (uint32_t a = 0; a < 4; ++a) {
                for (int i = 0; i < 3; ++i) set_outcome(E, s, a, i, 0.0, 0, 0.0, 0);
                char letter = map[row][col];
                if (letter == 'G' || letter == 'H') {
                    set_outcome(E, s, a, 0, 1.0, s, 0.0, 1);
                } else {
                    /* slippery: [(a-1)%4, a, (a+1)%4] with usize wrap (release): a=0 -> 3 */
                    uint32_t bs[3] = {(a + 3) % 4, a, (a + 1) % 4};
                    int nb = slippery ? 3 : 1;
                    for (int i = 0; i < nb; ++i) {
                        uint32_t b = slippery ? bs[i] : a;
                        uint32_t nr, nc;
                        inc(n, n, row, col, b, &nr, &nc);           /* update_probability_matrix :30-44 */
                        char nl = map[nr][nc];
                        int t = nl == 'G' || nl == 'H';
                        double r = nl == 'G' ? 1.0 : 0.0;
                        set_outcome(E, s, a, i, slippery ? 1.0 / 3.0 : 1.0, nr * n + nc, r, t);
                    }
                }
            }
        }
    E->trunc_reward = 0.0; /* frozen_lake.rs:119-122 */
}

/* FrozenLakeEditedEnv (src/env/frozen_lake_edited.rs).  Terrain of a cell
 * (get_terrain :146-162) and of the neighbour in direction a, WALL off the map
 * (get_obs :115-144); values (:18-28) feed the FL_OBS input adapter. */
enum { T_START = 0, T_WALL = 1, T_HOLE = 2, T_GROUND = 3, T_GOAL = 4 };
static int fl_terrain(const char **map, uint32_t row, uint32_t col) {
    switch (map[row][col]) {
    case 'S': return T_START;
    case 'G': return T_GOAL;
    case 'H': return T_HOLE;
    default: return T_GROUND;
    }
}
static int fl_neighbour(const char **map, uint32_t nrow, uint32_t ncol, uint32_t row, uint32_t col, uint32_t a) {
    switch (a) {
    case 0: return col == 0 ? T_WALL : fl_terrain(map, row, col - 1);
    case 1: return row == nrow - 1 ? T_WALL : fl_terrain(map, row + 1, col);
    case 2: return col == ncol - 1 ? T_WALL : fl_terrain(map, row, col + 1);
    default: return row == 0 ? T_WALL : fl_terrain(map, row - 1, col);
    }
}
static double fl_terrain_value(int t) {   /* FrozenLakeTerrain::value, frozen_lake_edited.rs:18-28 */
    switch (t) {
    case T_HOLE: return -1.0;
    case T_WALL: return -0.5;
    case T_START: return 0.0;
    case T_GROUND: return 0.5;
    default: return 1.0;
    }
}
/* FrozenLakeEditedEnv::new (:165-218) + update_probability_matrix (:94-113):
 * reward 10 for stepping onto G, else -1; terminated on G or H, judged by the
 * terrain in the moved direction; G/H rows are (1.0, s, 0.0, true). */
static void build_frozen_lake_edited(envdef *E, int map8, int slippery) {
    const char **map = map8 ? FL8 : FL4;
    uint32_t n = map8 ? 8 : 4;
    E->S = n * n; E->A = 4; E->nrow = E->ncol = n; E->map = map;
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < E->S; ++i) if (map[i / n][i % n] == 'S') cnt++;
    for (uint32_t i = 0; i < E->S; ++i) E->start[i] = map[i / n][i % n] == 'S' ? 1.0 / (double)cnt : 0.0;
    E->n_start = E->S;
    for (uint32_t row = 0; row < n; ++row)
        for (uint32_t col = 0; col < n; ++col) {
            uint32_t s = row * n + col;
            for (uint32_t a = 0; a < 4; ++a) {
                for (int i = 0; i < 3; ++i) set_outcome(E, s, a, i, 0.0, 0, 0.0, 0);
                char letter = map[row][col];
                if (letter == 'G' || letter == 'H') {
                    set_outcome(E, s, a, 0, 1.0, s, 0.0, 1);
                    continue;
                }
                uint32_t bs[3] = {(a + 3) % 4, a, (a + 1) % 4};   /* (a-1)%4 with usize wrap */
                int nb = slippery ? 3 : 1;
                for (int i = 0; i < nb; ++i) {
                    uint32_t b = slippery ? bs[i] : a;
                    int nt = fl_neighbour(map, n, n, row, col, b);
                    uint32_t nr, nc;
                    inc(n, n, row, col, b, &nr, &nc);
                    int win = nt == T_GOAL;
                    set_outcome(E, s, a, i, slippery ? 1.0 / 3.0 : 1.0, nr * n + nc, win ? 10.0 : -1.0,
                                win || nt == T_HOLE);
                }
            }
        }
    E->trunc_reward = -1.0;   /* step :227-231: (obs of the current position, -1.0, true) */
    E->trunc_stay = 1;
}

/* CliffWalkingEnv::new: src/env/cliff_walking.rs:22-58 */
static void build_cliff_walking(envdef *E) {
    E->S = 48; E->A = 4;
    for (uint32_t row = 0; row < 4; ++row)
        for (uint32_t col = 0; col < 12; ++col)
            for (uint32_t a = 0; a < 4; ++a) {
                uint32_t nr, nc;
                inc(4, 12, row, col, a, &nr, &nc);
                uint32_t ns = nr * 12 + nc;
                int win = ns == 47, lose = ns >= 37 && ns <= 46;
                for (int i = 0; i < 3; ++i) set_outcome(E, row * 12 + col, a, i, 0.0, 0, 0.0, 0);
                set_outcome(E, row * 12 + col, a, 0, 1.0, ns, lose ? -100.0 : -1.0, lose || win);
            }
    for (uint32_t i = 0; i < 48; ++i) E->start[i] = i == 36 ? 1.0 : 0.0;
    E->n_start = 48;
    E->trunc_reward = -100.0; /* cliff_walking.rs:81-84 */
}

/* TaxiEnv::new: src/env/taxi.rs:57-131 */
static void build_taxi(envdef *E) {
    E->S = 500; E->A = 6;
    double sum = 0.0;
    for (uint32_t i = 0; i < 500; ++i) E->start[i] = 0.0;
    for (uint32_t row = 0; row < 5; ++row)
        for (uint32_t col = 0; col < 5; ++col)
            for (uint32_t pass = 0; pass < 5; ++pass)
                for (uint32_t dest = 0; dest < 4; ++dest) {
                    uint32_t state = ((row * 5 + col) * 5 + pass) * 4 + dest;   /* encode :33-42 */
                    if (pass < 4 && pass != dest) { E->start[state] += 1.0; sum += 1.0; }
                    for (uint32_t action = 0; action < 6; ++action) {
                        uint32_t nrow = row, ncol = col, npass = pass;
                        double reward = -1.0;
                        int term = 0;
                        if (action == 0) nrow = row + 1 < 4 ? row + 1 : 4;
                        else if (action == 1) nrow = row != 0 ? row - 1 : 0;
                        if (action == 2 && TAXI_MAP[1 + row][2 * col + 2] == ':') {
                            ncol = col + 1 < 4 ? col + 1 : 4;
                        } else if (action == 3 && TAXI_MAP[1 + row][2 * col] == ':') {
                            ncol = col != 0 ? col - 1 : 0;
                        } else if (action == 4) {
                            if (pass < 4 && row == TAXI_LOCS[pass][0] && col == TAXI_LOCS[pass][1]) npass = 4;
                            else reward = -10.0;
                        } else if (action == 5) {
                            if (row == TAXI_LOCS[dest][0] && col == TAXI_LOCS[dest][1] && pass == 4) {
                                npass = dest; term = 1; reward = 20.0;
                            } else reward = -10.0;
                        }
                        uint32_t ns = ((nrow * 5 + ncol) * 5 + npass) * 4 + dest;
                        for (int i = 0; i < 3; ++i) set_outcome(E, state, action, i, 0.0, 0, 0.0, 0);
                        set_outcome(E, state, action, 0, 1.0, ns, reward, term);
                    }
                }
    for (uint32_t i = 0; i < 500; ++i) E->start[i] /= sum;    /* :117-119 */
    E->n_start = 500;
    E->trunc_reward = 0.0; /* taxi.rs:146-149 */
}

static int build_env_tables(envdef *E, const rlo_config *c) {
    switch (c->env) {
    case RLO_ENV_FROZEN_LAKE: build_frozen_lake(E, c->map8x8, c->slippery); return 0;
    case RLO_ENV_FROZEN_LAKE_EDITED: build_frozen_lake_edited(E, c->map8x8, c->slippery); return 0;
    case RLO_ENV_CLIFF_WALKING: build_cliff_walking(E); return 0;
    case RLO_ENV_TAXI: build_taxi(E); return 0;
    case RLO_ENV_BLACKJACK: E->S = 32 * 32 * 2; E->A = 2; return 0;
    }
    return -1;
}
static int build_env(envdef *E, const rlo_config *c) {
    memset(E, 0, sizeof(*E));
    E->kind = c->env;
    E->max_steps = c->max_steps;
    if (build_env_tables(E, c)) return -1;
    E->slippery = c->slippery != 0;
    /* one state of probability 1: categorical_sample (utils.rs:33-43) returns it for every u */
    uint32_t nz = 0, at = 0;
    for (uint32_t i = 0; i < E->n_start; ++i)
        if (E->start[i] != 0.0) { nz++; at = i; }
    E->fixed_start = (nz == 1 && E->start[at] == 1.0) ? (int32_t)at : -1;
    return 0;
}

int rlo_env_dims(const rlo_config *c, uint32_t *S, uint32_t *A) {
    static envdef E;
    if (build_env(&E, c)) return -1;
    *S = E.S; *A = E.A;
    return 0;
}
int rlo_env_table(const rlo_config *c, double *prob, uint32_t *next, double *reward, uint8_t *term) {
    static envdef E;
    if (build_env(&E, c) || c->env == RLO_ENV_BLACKJACK) return -1;
    size_t n = (size_t)E.S * E.A * 3;
    memcpy(prob, E.prob, n * sizeof(double));
    memcpy(next, E.next, n * sizeof(uint32_t));
    memcpy(reward, E.rew, n * sizeof(double));
    memcpy(term, E.term, n);
    return 0;
}
int rlo_env_start(const rlo_config *c, double *start) {
    static envdef E;
    if (build_env(&E, c) || c->env == RLO_ENV_BLACKJACK) return -1;
    memcpy(start, E.start, E.S * sizeof(double));
    return 0;
}

/* blackjack helpers: src/env/blackjack.rs:47-83 */
static inline uint32_t bj_score(uint32_t sum, uint32_t ace) { return (ace && sum + 10 <= 21) ? sum + 10 : sum; }
/* dense obs index: p_score <= 31, d_score <= 26 (dealer stops at >= 17) */
static inline uint32_t bj_index(uint32_t p, uint32_t d, uint32_t ace) { return (p * 32 + d) * 2 + (ace ? 1 : 0); }
static void bj_initialize_hands(envstate *st, rlo_rng *r) {       /* :47-56 */
    cardsrc cs = {0, 0};
    uint32_t p0 = draw_card(r, &cs), p1 = draw_card(r, &cs), d0 = draw_card(r, &cs), d1 = draw_card(r, &cs);
    st->p_sum = p0 + p1; st->d_sum = d0 + d1; st->d0 = d0;
    st->p_ace = p0 == 1 || p1 == 1;
    st->d_ace = d0 == 1 || d1 == 1;
}

/* Env::reset: frozen_lake.rs:106-113, cliff_walking.rs:70-75, taxi.rs:135-142, blackjack.rs:105-116 */
static uint32_t env_reset(const envdef *E, envstate *st, rlo_rng *r) {
    if (E->kind == RLO_ENV_BLACKJACK) {
        bj_initialize_hands(st, r);
        st->ready = 1;
        return bj_index(bj_score(st->p_sum, st->p_ace), st->d0, st->p_ace);
    }
    if (E->kind == RLO_ENV_CLIFF_WALKING) {
        st->pos = 36;
    } else if (E->fixed_start >= 0) {
        /* one start state (FrozenLake's maps): categorical_sample returns it for
         * every u, so the reference's draw (frozen_lake.rs:107-108) is not made */
        st->pos = (uint32_t)E->fixed_start;
    } else {
        double u = uniform01(r);
        st->pos = categorical_sample(E->start, E->n_start, u);
    }
    st->ready = 1;
    st->curr_step = 0;
    return st->pos;
}

/* Env::step: frozen_lake.rs:115-134, cliff_walking.rs:77-91, taxi.rs:144-159,
 * blackjack.rs:118-163.  Returns -1 (EnvNotReady) if not ready. */
static int env_step(const envdef *E, envstate *st, uint32_t a, rlo_rng *r, uint32_t *s2, double *rew,
                    int *term) {
    if (!st->ready) return -1;
    if (E->kind == RLO_ENV_BLACKJACK) {
        if (a == 0) {                                   /* hit :121-138 */
            cardsrc cs = {0, 0};
            st->p_sum += draw_card(r, &cs);
            uint32_t p = bj_score(st->p_sum, st->p_ace);
            if (p > 21) {
                st->ready = 0;
                *s2 = bj_index(p, bj_score(st->d_sum, st->d_ace), st->p_ace);
                *rew = -1.0; *term = 1;
                return 0;
            }
            *s2 = bj_index(p, st->d0, st->p_ace);
            *rew = 0.0; *term = 0;
            return 0;
        }
        st->ready = 0;                                  /* stick :139-162 */
        uint32_t d = bj_score(st->d_sum, st->d_ace);
        cardsrc cs = {0, 0};
        while (d < 17) {
            st->d_sum += draw_card(r, &cs);
            d = bj_score(st->d_sum, st->d_ace);
        }
        uint32_t p = bj_score(st->p_sum, st->p_ace);
        *s2 = bj_index(p, d, st->p_ace);
        *term = 1;
        if (d > 21) *rew = 1.0;
        else *rew = p > d ? 1.0 : (p < d ? -1.0 : 0.0);
        return 0;
    }
    if (st->curr_step >= E->max_steps) {            /* truncation: (0 | pos, r_trunc, true) */
        st->ready = 0;
        *s2 = E->trunc_stay ? st->pos : 0; *rew = E->trunc_reward; *term = 1;
        return 0;
    }
    st->curr_step += 1;
    size_t k = ((size_t)st->pos * E->A + a) * 3;
    uint32_t i = 0;
    if ((E->kind == RLO_ENV_FROZEN_LAKE || E->kind == RLO_ENV_FROZEN_LAKE_EDITED) && E->slippery) {
        /* the reference draws here on deterministic maps too (frozen_lake.rs:126),
         * a value categorical_sample([1, 0, 0]) ignores: not made there */
        double u = uniform01(r);
        i = categorical_sample(&E->prob[k], 3, u);
    }
    st->pos = E->next[k + i];
    *s2 = st->pos; *rew = E->rew[k + i]; *term = E->term[k + i];
    if (*term) st->ready = 0;
    return 0;
}

int rlo_env_walk(const rlo_config *c, uint64_t lane, uint32_t n, const uint32_t *actions, uint32_t *s0,
                 uint32_t *s_next, double *reward, uint8_t *term) {
    static envdef E;
    if (build_env(&E, c)) return -1;
    envstate st;
    rlo_rng r;
    memset(&st, 0, sizeof st);
    rng_seed(&r, c->seed, lane);
    if (c->env == RLO_ENV_BLACKJACK) bj_initialize_hands(&st, &r);
    *s0 = env_reset(&E, &st, &r);
    for (uint32_t i = 0; i < n; ++i) {
        int tm = 0;
        if (env_step(&E, &st, actions[i], &r, &s_next[i], &reward[i], &tm)) return (int)i;
        term[i] = (uint8_t)tm;
    }
    return (int)n;
}

/* ======================================================================== */
/* action selection & TD targets (shared by both restatements)              */
/* ======================================================================== */
/* UpperConfidenceBound ucbs: upper_confidence_bound.rs:29-37,53-57 */
static inline double ucb_value(double q, double c, double lnt, double n) {
    return q + c * sqrt(lnt / (n + MIN_POSITIVE));
}
/* UniformEpsilonGreed::get_exploration_probs: uniform_epsilon_greed.rs:72-76 */
static void eps_probs(double eps, const double *q, uint32_t A, double *p) {
    for (uint32_t i = 0; i < A; ++i) p[i] = eps / (double)A;
    p[argmax_d(q, A)] = 1.0 - eps;
}
/* UCB get_exploration_probs: upper_confidence_bound.rs:48-63 */
static void ucb_probs(const double *q, const uint64_t *n, uint64_t t, double c, uint32_t A, double *p) {
    double lnt = rlo_log((double)t);
    double sum = 0.0;
    for (uint32_t i = 0; i < A; ++i) {
        p[i] = ucb_value(q[i], c, lnt, (double)n[i]);
        sum += p[i];
    }
    for (uint32_t i = 0; i < A; ++i) p[i] /= sum;
}
/* sarsa / qlearning / expected_sarsa: src/agent.rs:19-45 */
static double future_q(int algo, const double *q2, uint32_t a2, const double *p, uint32_t A) {
    if (algo == RLO_ALGO_SARSA) return q2[a2];
    if (algo == RLO_ALGO_QLEARNING) return max_d(q2, A);
    double f = 0.0;
    for (uint32_t i = 0; i < A; ++i) f += p[i] * q2[i];
    return f;
}
/* decay_epsilon: uniform_epsilon_greed.rs:42-49 with the bins' closure
 * `a - epsilon_decay` (src/bin/frozen_lake.rs:84,146) or `a * d` (frozen_lake_neural.rs:181) */
static double decay_eps(const rlo_config *c, double eps) {
    double nw = c->decay_kind == RLO_DECAY_MUL ? eps * c->eps_decay : eps - c->eps_decay;
    return c->eps_final > nw ? eps : nw;
}

/* ======================================================================== */
/* NeuralPolicy over Network (src/policy/neural_policy.rs, src/network.rs,   */
/* src/network/{layers,activation,loss}.rs).  Shape of the neural bin        */
/* (src/bin/frozen_lake_neural.rs:130-134): DenseLayer(n_in, H) -> act1 ->   */
/* DenseLayer(H, A) -> act2, mse.  Parameters [W1 n_in x H][b1 H][W2 H x A]  */
/* [b2 A].  ndarray's dot (matrixmultiply dgemm) accumulates every output    */
/* element over k in order from 0.0; that order is restated here WITHOUT      */
/* fused multiply-add (dgemm's FMA use depends on the host CPU: parity with   */
/* the Rust binary is unpinned; the GPU matches this restatement bit for bit).*/
/* ======================================================================== */
typedef struct { uint32_t in, H, A, np; int act1, act2; } netdef;
static double max_rs(double a, double b) { return (a > b || b != b) ? a : b; }   /* f64::max */
static double min_rs(double a, double b) { return (a < b || b != b) ? a : b; }   /* f64::min */
static double sigmoid_(double v) { return 1.0 / (1.0 + rlo_exp(-v)); }
/* activation.rs:5-94, elementwise pairs (softmax is layer-wide, see below) */
static double act_f(int act, double v) {
    switch (act) {
    case RLO_ACT_TANH: return rlo_tanh(v);                                       /* :15-17 */
    case RLO_ACT_RELU: return max_rs(v, 0.0);                                    /* :23-25 */
    case RLO_ACT_LEAKY_RELU: return max_rs(v, 0.1 * v);                          /* :31-33 */
    case RLO_ACT_RELU6: return min_rs(max_rs(v, 0.0), 6.0);                      /* :39-41 */
    case RLO_ACT_LEAKY_RELU6: return min_rs(max_rs(v, 0.1 * v), 6.0);            /* :47-49 */
    case RLO_ACT_SIGMOID: return sigmoid_(v);                                    /* :55-57 */
    case RLO_ACT_SWISH: return v * sigmoid_(v);                                  /* :76-78 */
    case RLO_ACT_HARD_SWISH: return (v * min_rs(max_rs(v + 3.0, 0.0), 6.0)) / 6.0; /* :84-86 */
    default: return v;                                                           /* linear :7-9 */
    }
}
static double act_fp(int act, double v) {
    switch (act) {
    case RLO_ACT_TANH: { double t = rlo_tanh(v); return 1.0 - t * t; }          /* :19-21 powf(2.0) */
    case RLO_ACT_RELU: return v > 0.0 ? 1.0 : 0.0;                              /* :27-29 */
    case RLO_ACT_LEAKY_RELU: return v > 0.0 ? 1.0 : 0.01;                       /* :35-37 */
    case RLO_ACT_RELU6: return (v > 0.0 && v < 6.0) ? 1.0 : 0.0;                /* :43-45 */
    case RLO_ACT_LEAKY_RELU6: return (v > 0.0 && v < 6.0) ? 1.0 : 0.01;         /* :51-53 */
    case RLO_ACT_SIGMOID: { double sg = sigmoid_(v); return sg * (1.0 - sg); }  /* :59-62 */
    case RLO_ACT_SWISH: {                                                       /* :80-82 */
        double e = rlo_exp(v);
        return (e * (v + e + 1.0)) / ((e + 1.0) * (e + 1.0));
    }
    case RLO_ACT_HARD_SWISH: return v > -3.0 ? (2.0 * v + 3.0) / 6.0 : 0.0;    /* :88-94 */
    default: return 1.0;                                                        /* linear :11-13 */
    }
}
void rlo_act(int32_t act, double x, double *f, double *fp) { *f = act_f(act, x); *fp = act_fp(act, x); }
/* softmax (:64-74): e = exp(v - ndarray_max(v)) (utils.rs:23-31, strict >), e / e.sum();
 * ndarray's sum is its eightfold unrolled fold (8 partial sums, then the tail).
 * softmax_prime is the same function (as written, :70-74). */
static void softmax_(const double *v, uint32_t n, double *out) {
    double m = v[0], e[MAXA], acc = 0.0;
    for (uint32_t i = 0; i < n; ++i) if (v[i] > m) m = v[i];
    for (uint32_t i = 0; i < n; ++i) e[i] = rlo_exp(v[i] - m);
    /* n = COUNT <= 6 < 8: the unrolled fold's partial sums stay 0.0 and the sum is
     * the sequential tail 0.0 + e0 + e1 + ... */
    for (uint32_t i = 0; i < n; ++i) acc = acc + e[i];
    for (uint32_t k = 0; k < n; ++k) out[k] = e[k] / acc;
}
static void act_layer(int act, const double *v, uint32_t n, double *out) {
    if (act == RLO_ACT_SOFTMAX) { softmax_(v, n, out); return; }
    for (uint32_t i = 0; i < n; ++i) out[i] = act_f(act, v[i]);
}
static void act_layer_prime(int act, const double *v, uint32_t n, double *out) {
    if (act == RLO_ACT_SOFTMAX) { softmax_(v, n, out); return; }
    for (uint32_t i = 0; i < n; ++i) out[i] = act_fp(act, v[i]);
}

static int net_make(const rlo_config *c, uint32_t A, netdef *n) {
    if (c->policy != RLO_POLICY_NEURAL) return -1;
    n->in = c->net_input == RLO_INPUT_FL_OBS ? 6u : 1u;
    n->H = c->net_hidden; n->A = A; n->act1 = c->net_act1; n->act2 = c->net_act2;
    if (n->H == 0 || n->H > 256 || n->act1 == RLO_ACT_SOFTMAX || n->act1 < 0 || n->act1 > 9 ||
        n->act2 < 0 || n->act2 > 9)
        return -1;
    if (c->net_input == RLO_INPUT_FL_OBS && c->env != RLO_ENV_FROZEN_LAKE && c->env != RLO_ENV_FROZEN_LAKE_EDITED)
        return -1;
    if (c->net_input == RLO_INPUT_SCALAR && c->env == RLO_ENV_FROZEN_LAKE_EDITED) return -1; /* struct obs */
    n->np = n->in * n->H + n->H + n->H * A + A;
    return 0;
}
/* input adapters: [[obs as f64]] (frozen_lake_neural.rs:147-149) of the reference
 * observation id, or the FrozenLakeObs features (:136-145) */
static void net_features(const envdef *E, const netdef *n, int input, double *feat) {
    for (uint32_t s = 0; s < E->S; ++s) {
        double *x = feat + (size_t)s * n->in;
        if (input == RLO_INPUT_FL_OBS) {
            uint32_t row = s / E->ncol, col = s % E->ncol;
            for (uint32_t a = 0; a < 4; ++a)
                x[a] = fl_terrain_value(fl_neighbour(E->map, E->nrow, E->ncol, row, col, a));
            x[4] = (double)row;
            x[5] = (double)col;
        } else if (E->kind == RLO_ENV_BLACKJACK) {
            x[0] = (double)rlo_blackjack_obs_id(s >> 6, (s >> 1) & 31u, s & 1u);
        } else {
            x[0] = (double)s;
        }
    }
}
/* forward: opre = pre-activation output layer, y = act2(opre).  Dense: x.dot(W) + b
 * (layers.rs:78-81); Activation: f(input) (:130-133) */
static void net_forward(const netdef *n, const double *w, const double *x, double *opre, double *y) {
    const double *W1 = w, *b1 = w + n->in * n->H, *W2 = b1 + n->H, *b2 = W2 + (size_t)n->H * n->A;
    double acc[MAXA];
    for (uint32_t i = 0; i < n->A; ++i) acc[i] = 0.0;
    for (uint32_t j = 0; j < n->H; ++j) {
        double z = 0.0;
        for (uint32_t k = 0; k < n->in; ++k) z = z + x[k] * W1[(size_t)k * n->H + j];
        z = z + b1[j];
        double h = act_f(n->act1, z);
        for (uint32_t i = 0; i < n->A; ++i) acc[i] = acc[i] + h * W2[(size_t)j * n->A + i];
    }
    for (uint32_t i = 0; i < n->A; ++i) opre[i] = acc[i] + b2[i];
    act_layer(n->act2, opre, n->A, y);
}
/* Network::fit (src/network.rs:61-80): forward, error = mse_prime (loss.rs:4-9:
 * 2*(y_pred - y_true)/len), then backward through the layers in reverse
 * (layers.rs:83-93, :135-141): Dense input_error = err.dot(W.t()) with the old W,
 * W -= lr * input.t().dot(err), b -= lr * err. */
static void net_fit(const netdef *n, double *w, const double *x, const double *target, double lr) {
    double *W1 = w, *b1 = w + n->in * n->H, *W2 = b1 + n->H, *b2 = W2 + (size_t)n->H * n->A;
    double opre[MAXA], y[MAXA], pr[MAXA], e2[MAXA];
    net_forward(n, w, x, opre, y);
    act_layer_prime(n->act2, opre, n->A, pr);
    for (uint32_t i = 0; i < n->A; ++i) e2[i] = pr[i] * ((2.0 * (y[i] - target[i])) / (double)n->A);
    for (uint32_t j = 0; j < n->H; ++j) {
        double z = 0.0;
        for (uint32_t k = 0; k < n->in; ++k) z = z + x[k] * W1[(size_t)k * n->H + j];
        z = z + b1[j];
        const double h = act_f(n->act1, z);
        double ie = 0.0;
        for (uint32_t i = 0; i < n->A; ++i) ie = ie + e2[i] * W2[(size_t)j * n->A + i];
        for (uint32_t i = 0; i < n->A; ++i) {
            double *wv = &W2[(size_t)j * n->A + i];
            *wv = *wv - lr * (0.0 + h * e2[i]);
        }
        const double e1 = act_fp(n->act1, z) * ie;
        for (uint32_t k = 0; k < n->in; ++k) {
            double *wv = &W1[(size_t)k * n->H + j];
            *wv = *wv - lr * (0.0 + x[k] * e1);
        }
        b1[j] = b1[j] - lr * e1;
    }
    for (uint32_t i = 0; i < n->A; ++i) b2[i] = b2[i] - lr * e2[i];
}
/* rand 0.8.5 UniformFloat::<f64>::new(low, high) scale (decrease until
 * scale * max_rand + low < high) */
static double uniform_scale(double low, double high) {
    const double max_rand = 1.0 - 0x1p-52;
    double scale = high - low;
    while (scale * max_rand + low >= high) { dbits b; b.d = scale; b.u -= 1; scale = b.d; }
    return scale;
}
/* weight stream of generation `gen` (0 = DenseLayer::new, k = the k-th Network::reset) */
static uint64_t net_seed(uint64_t seed, uint32_t gen) { return seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(gen + 1u)); }
/* DenseLayer::new (layers.rs:55-73): W ~ Uniform::new(-l, l), l = sqrt(6/(in+out)),
 * drawn row-major, b = 0; DenseLayer::reset (:90-95): new W the same way, b = 0.1 */
static void net_init(const netdef *n, double *w, uint64_t seed, uint64_t lane, uint32_t gen) {
    rlo_rng r;
    rng_seed(&r, net_seed(seed, gen), lane);
    const uint32_t dims[2][2] = {{n->in, n->H}, {n->H, n->A}};
    double *p = w;
    for (int L = 0; L < 2; ++L) {
        const uint32_t fi = dims[L][0], fo = dims[L][1];
        const double l = sqrt(6.0 / (double)(fi + fo));
        const double scale = uniform_scale(-l, l);
        for (uint32_t k = 0; k < fi * fo; ++k) {
            dbits b; b.u = (next_u64(&r) >> 12) | 0x3FF0000000000000ull;
            p[k] = (b.d - 1.0) * scale + -l;
        }
        p += fi * fo;
        for (uint32_t k = 0; k < fo; ++k) p[k] = gen ? 0.1 : 0.0;
        p += fo;
    }
}
int rlo_net_dims(const rlo_config *c, uint32_t *n_in, uint32_t *n_params) {
    envdef *E = (envdef *)malloc(sizeof(envdef));
    netdef n;
    int rc = build_env(E, c) || net_make(c, E->A, &n) ? -1 : 0;
    if (!rc) { *n_in = n.in; *n_params = n.np; }
    free(E);
    return rc;
}
int rlo_net_features(const rlo_config *c, double *out) {
    envdef *E = (envdef *)malloc(sizeof(envdef));
    netdef n;
    int rc = build_env(E, c) || net_make(c, E->A, &n) ? -1 : 0;
    if (!rc) net_features(E, &n, c->net_input, out);
    free(E);
    return rc;
}
void rlo_net_init(const rlo_config *c, uint64_t lane, uint32_t gen, double *w) {
    envdef *E = (envdef *)malloc(sizeof(envdef));
    netdef n;
    if (!build_env(E, c) && !net_make(c, E->A, &n)) net_init(&n, w, c->seed, lane, gen);
    free(E);
}
void rlo_net_forward(const rlo_config *c, const double *w, const double *x, double *y) {
    envdef *E = (envdef *)malloc(sizeof(envdef));
    netdef n;
    double opre[MAXA];
    if (!build_env(E, c) && !net_make(c, E->A, &n)) net_forward(&n, w, x, opre, y);
    free(E);
}
void rlo_net_fit(const rlo_config *c, double *w, const double *x, const double *y_target, double lr) {
    envdef *E = (envdef *)malloc(sizeof(envdef));
    netdef n;
    if (!build_env(E, c) && !net_make(c, E->A, &n)) net_fit(&n, w, x, y_target, lr);
    free(E);
}

/* ======================================================================== */
/* 1. faithful single-env restatement                                        */
/* ======================================================================== */
typedef struct { void *p; size_t n, cap, esz; } vec;
static void vpush(vec *v, const void *x) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 1024;
        v->p = realloc(v->p, v->cap * v->esz);
    }
    memcpy((char *)v->p + v->n * v->esz, x, v->esz);
    v->n++;
}

struct rlo_faithful {
    rlo_config c;
    envdef E;
    envstate st;
    rlo_rng rng;
    uint32_t S, A, P;
    double *q;           /* [P][S][A] f64 */
    int dflag;           /* DoubleTabularPolicy::policy_flag (starts true) */
    double eps;
    uint64_t *ucb_n;     /* [S][A] (u128 in the reference) */
    uint64_t ucb_t;
    double *trace;       /* [S][A] */
    uint8_t *visited;    /* [S] — membership of the trace FxHashMap */
    uint32_t *vlist, vcnt; /* visited states in first-visit order (the sweep order, see f_update) */
    netdef net;          /* NeuralPolicy */
    double *w, *feat;    /* parameters [np], input features [S][in] */
    uint32_t net_gen;    /* Network::reset calls so far */
    vec reward_history, episode_length, training_error, records;
    int record;
    uint32_t plan;       /* InternalModelAgent planning steps (0: plain agent) */
    model_t model;
};

static void f_clear_policy(rlo_faithful *f) {
    if (f->w) { net_init(&f->net, f->w, f->c.seed, f->c.lane_offset, ++f->net_gen); return; }  /* Network::reset */
    for (size_t i = 0; i < (size_t)f->P * f->S * f->A; ++i) f->q[i] = f->c.q_default;
}
static void f_reset_selector(rlo_faithful *f) {
    f->eps = f->c.eps0;
    memset(f->ucb_n, 0, sizeof(uint64_t) * f->S * f->A);
    f->ucb_t = 1;
}

rlo_faithful *rlo_faithful_create(const rlo_config *c) {
    rlo_faithful *f = (rlo_faithful *)calloc(1, sizeof(rlo_faithful));
    f->c = *c;
    if (build_env(&f->E, c)) { free(f); return NULL; }
    f->S = f->E.S; f->A = f->E.A; f->P = c->policy == RLO_POLICY_DOUBLE ? 2 : 1;
    f->q = (double *)malloc(sizeof(double) * f->P * f->S * f->A);
    f->ucb_n = (uint64_t *)calloc((size_t)f->S * f->A, sizeof(uint64_t));
    f->trace = (double *)calloc((size_t)f->S * f->A, sizeof(double));
    f->visited = (uint8_t *)calloc(f->S, 1);
    f->vlist = (uint32_t *)calloc(f->S, sizeof(uint32_t));
    if (c->policy == RLO_POLICY_NEURAL) {
        if (net_make(c, f->A, &f->net)) { free(f->q); free(f->ucb_n); free(f->trace); free(f->visited); free(f->vlist); free(f); return NULL; }
        f->w = (double *)malloc(sizeof(double) * f->net.np);
        f->feat = (double *)malloc(sizeof(double) * f->S * f->net.in);
        net_features(&f->E, &f->net, c->net_input, f->feat);
    }
    f->reward_history.esz = sizeof(double);
    f->episode_length.esz = sizeof(uint64_t);
    f->training_error.esz = sizeof(double);
    f->records.esz = sizeof(rlo_record);
    f->dflag = 1;
    if (f->w) net_init(&f->net, f->w, c->seed, c->lane_offset, 0);   /* NeuralPolicy::new */
    else f_clear_policy(f);
    f_reset_selector(f);
    rng_seed(&f->rng, c->seed, c->lane_offset);
    if (c->env == RLO_ENV_BLACKJACK) bj_initialize_hands(&f->st, &f->rng); /* BlackJackEnv::new deals */
    return f;
}
void rlo_faithful_destroy(rlo_faithful *f) {
    if (!f) return;
    free(f->q); free(f->ucb_n); free(f->trace); free(f->visited); free(f->vlist); free(f->w); free(f->feat);
    free(f->reward_history.p); free(f->episode_length.p); free(f->training_error.p); free(f->records.p);
    model_free(&f->model);
    free(f);
}
void rlo_faithful_set_record(rlo_faithful *f, int e) { f->record = e; }
double rlo_faithful_epsilon(const rlo_faithful *f) { return f->eps; }

/* Policy::predict: tabular_policy.rs:27-29, double_tabular_policy.rs:31-40,
 * neural_policy.rs:43-47 (input adapter, Network::predict, output adapter) */
static void f_predict(const rlo_faithful *f, uint32_t s, double *out) {
    if (f->w) { double opre[MAXA]; net_forward(&f->net, f->w, f->feat + (size_t)s * f->net.in, opre, out); return; }
    const double *a = &f->q[(size_t)s * f->A];
    if (f->P == 1) { for (uint32_t i = 0; i < f->A; ++i) out[i] = a[i]; return; }
    const double *b = &f->q[((size_t)f->S + s) * f->A];
    for (uint32_t i = 0; i < f->A; ++i) out[i] = (a[i] + b[i]) / 2.0;
}
/* Policy::get_values: tabular_policy.rs:31-33, double_tabular_policy.rs:42-50 (flag ? alpha : beta),
 * neural_policy.rs:49-53 */
static void f_values(const rlo_faithful *f, uint32_t s, double *out) {
    if (f->w) { f_predict(f, s, out); return; }
    uint32_t tbl = (f->P == 2 && !f->dflag) ? 1 : 0;
    memcpy(out, &f->q[((size_t)tbl * f->S + s) * f->A], f->A * sizeof(double));
}
/* Policy::update: tabular_policy.rs:35-38, double_tabular_policy.rs:52-60 (flag ? beta : alpha);
 * neural_policy.rs:55-62: y = get_values(s), y[a] += td, Network::fit(x(s), y, lr) */
static void f_policy_update(rlo_faithful *f, uint32_t s, uint32_t a, double td) {
    if (f->w) {
        double y[MAXA];
        f_values(f, s, y);
        y[a] += td;
        net_fit(&f->net, f->w, f->feat + (size_t)s * f->net.in, y, f->c.lr);
        return;
    }
    uint32_t tbl = (f->P == 2 && f->dflag) ? 1 : 0;
    f->q[((size_t)tbl * f->S + s) * f->A + a] += f->c.lr * td;
}
/* Agent::get_action: one_step_agent.rs:48-51 / elegibility_traces_agent.rs:56-59 */
static uint32_t f_get_action(rlo_faithful *f, uint32_t s) {
    double v[MAXA];
    f_predict(f, s, v);
    if (f->c.selector == RLO_SEL_EPS_GREEDY) {             /* uniform_epsilon_greed.rs:60-66 */
        if (f->eps != 0.0 && eps_test(&f->rng, f->eps)) return uniform_action(&f->rng, f->A);
        return argmax_d(v, f->A);
    }
    uint64_t *n = &f->ucb_n[(size_t)s * f->A];             /* upper_confidence_bound.rs:29-42 */
    double lnt = rlo_log((double)f->ucb_t);
    double u[MAXA];
    for (uint32_t i = 0; i < f->A; ++i) u[i] = ucb_value(v[i], f->c.ucb_c, lnt, (double)n[i]);
    uint32_t a = argmax_d(u, f->A);
    n[a] += 1;
    f->ucb_t += 1;
    return a;
}
/* Agent::update: one_step_agent.rs:53-86 and elegibility_traces_agent.rs:61-104 */
static double f_update(rlo_faithful *f, uint32_t s, uint32_t a, double r, int term, uint32_t s2,
                       uint32_t a2) {
    const uint32_t A = f->A;
    double q2[MAXA], p[MAXA], q[MAXA];
    f_values(f, s2, q2);
    if (f->c.selector == RLO_SEL_EPS_GREEDY) eps_probs(f->eps, q2, A, p);
    else ucb_probs(q2, &f->ucb_n[(size_t)s2 * A], f->ucb_t, f->c.ucb_c, A, p);
    double fq = future_q(f->c.algo, q2, a2, p, A);
    f_values(f, s, q);
    double td = r + f->c.gamma * fq - q[a];
    if (f->c.agent == RLO_AGENT_ONE_STEP) {
        f_policy_update(f, s, a, td);
    } else {
        f->trace[(size_t)s * A + a] += 1.0;
        if (!f->visited[s]) { f->visited[s] = 1; f->vlist[f->vcnt++] = s; }
        /* the reference sweeps its FxHashMap; tabular updates are order-free, the
         * neural policy's are not: the sweep runs in first-visit order (as the GPU) */
        for (uint32_t vi = 0; vi < f->vcnt; ++vi) {
            const uint32_t o = f->vlist[vi];
            for (uint32_t b = 0; b < A; ++b) {
                double *e = &f->trace[(size_t)o * A + b];
                f_policy_update(f, o, b, td * *e);
                *e *= f->c.gamma * f->c.lambda_;
            }
        }
    }
    if (f->P == 2) f->dflag = !f->dflag;                   /* after_update */
    if (term) {
        if (f->c.agent == RLO_AGENT_TRACES) {
            memset(f->trace, 0, sizeof(double) * f->S * A);
            memset(f->visited, 0, f->S);
            f->vcnt = 0;
        }
        if (f->c.selector == RLO_SEL_EPS_GREEDY) f->eps = decay_eps(&f->c, f->eps);
    }
    return td;
}

/* InternalModelAgent::update (src/agent/internal_model_agent.rs:47-77): the inner
 * update, then model.add_info, then planning_steps replays of a uniformly drawn
 * model entry through the inner get_action + update(terminated = false). */
static double f_agent_update(rlo_faithful *f, uint32_t s, uint32_t a, double r, int term, uint32_t s2,
                             uint32_t a2) {
    double td = f_update(f, s, a, r, term, s2, a2);
    if (!f->plan) return td;
    model_add(&f->model, s * f->A + a, s2, r);
    for (uint32_t i = 0; i < f->plan; ++i) {
        uint32_t j = gen_index(&f->rng, f->model.cnt);
        uint32_t k = f->model.key[j], ps = k / f->A, pa = k % f->A, ps2 = f->model.s2[j];
        double pr = f->model.r[j];
        uint32_t na = f_get_action(f, ps2);
        f_update(f, ps, pa, pr, 0, ps2, na);
    }
    return td;
}
void rlo_faithful_set_planning(rlo_faithful *f, uint32_t planning_steps) {
    model_free(&f->model);
    f->plan = planning_steps;
    if (planning_steps) model_alloc(&f->model, (size_t)f->S * f->A);
}

/* Agent::evaluate: src/agent.rs:120-141 */
uint64_t rlo_faithful_evaluate(rlo_faithful *f, uint64_t n_episodes) {
    uint64_t steps = 0;
    for (uint64_t ep = 0; ep < n_episodes; ++ep) {
        uint32_t a = f_get_action(f, env_reset(&f->E, &f->st, &f->rng));
        for (;;) {
            uint32_t s2; double r; int term;
            if (env_step(&f->E, &f->st, a, &f->rng, &s2, &r, &term)) abort(); /* unwrap */
            steps++;
            a = f_get_action(f, s2);
            if (term) break;
        }
    }
    return steps;
}

/* Agent::train: src/agent.rs:66-118 */
uint64_t rlo_faithful_train(rlo_faithful *f, uint64_t n_episodes, uint64_t eval_at) {
    f->reward_history.n = f->episode_length.n = f->training_error.n = f->records.n = 0;
    uint64_t steps = 0;
    for (uint64_t episode = 0; episode < n_episodes; ++episode) {
        uint64_t action_counter = 0;
        double epi_reward = 0.0;
        uint32_t s = env_reset(&f->E, &f->st, &f->rng);
        uint32_t a = f_get_action(f, s);
        for (;;) {
            action_counter++;
            uint32_t s2; double r; int term;
            if (env_step(&f->E, &f->st, a, &f->rng, &s2, &r, &term)) abort();
            uint32_t a2 = f_get_action(f, s2);
            double td = f_agent_update(f, s, a, r, term, s2, a2);
            vpush(&f->training_error, &td);
            if (f->record) {
                rlo_record rec;
                memset(&rec, 0, sizeof rec);
                rec.s = s; rec.a = (uint8_t)a; rec.s2 = s2; rec.a2 = (uint8_t)a2;
                rec.r = r; rec.term = (uint8_t)term; rec.td = td; rec.mode = RLO_MODE_TRAIN;
                vpush(&f->records, &rec);
            }
            steps++;
            s = s2; a = a2;
            epi_reward += r;
            if (term) { vpush(&f->reward_history, &epi_reward); break; }
        }
        if (eval_at && episode % eval_at == 0) rlo_faithful_evaluate(f, f->c.eval_episodes);
        vpush(&f->episode_length, &action_counter);
    }
    return steps;
}
/* Agent::reset (one_step_agent.rs:43-46): selector.reset + policy.reset (flag kept) */
void rlo_faithful_reset(rlo_faithful *f) { f_reset_selector(f); f_clear_policy(f); f->model.cnt = 0; }
void rlo_faithful_get_q(const rlo_faithful *f, double *out) {
    if (f->w) { for (uint32_t s = 0; s < f->S; ++s) f_values(f, s, out + (size_t)s * f->A); return; }
    memcpy(out, f->q, sizeof(double) * f->P * f->S * f->A);
}
void rlo_faithful_get_weights(const rlo_faithful *f, double *out) {
    if (f->w) memcpy(out, f->w, sizeof(double) * f->net.np);
}
void rlo_faithful_set_weights(rlo_faithful *f, const double *in) {
    if (f->w) memcpy(f->w, in, sizeof(double) * f->net.np);
}
uint64_t rlo_faithful_n_episodes(const rlo_faithful *f) { return f->reward_history.n; }
uint64_t rlo_faithful_n_steps(const rlo_faithful *f) { return f->training_error.n; }
void rlo_faithful_histories(const rlo_faithful *f, double *rh, uint64_t *el, double *te) {
    /* memcpy with a null pointer is undefined even for 0 bytes (UBSan) */
    if (rh && f->reward_history.n) memcpy(rh, f->reward_history.p, f->reward_history.n * sizeof(double));
    if (el && f->episode_length.n) memcpy(el, f->episode_length.p, f->episode_length.n * sizeof(uint64_t));
    if (te && f->training_error.n) memcpy(te, f->training_error.p, f->training_error.n * sizeof(double));
}
uint64_t rlo_faithful_get_records(const rlo_faithful *f, rlo_record *out, uint64_t cap) {
    uint64_t n = f->records.n < cap ? f->records.n : cap;
    if (n) memcpy(out, f->records.p, n * sizeof(rlo_record));
    return f->records.n;
}
uint64_t rlo_faithful_bench(const rlo_config *c, uint64_t n_episodes, uint64_t eval_at, double *sec) {
    rlo_faithful *f = rlo_faithful_create(c);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    uint64_t steps = rlo_faithful_train(f, n_episodes, eval_at);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    *sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    rlo_faithful_destroy(f);
    return steps;
}

/* ======================================================================== */
/* 2. batched schedule (the GPU semantics)                                   */
/*                                                                           */
/* Per learner group g (lanes [g*G, (g+1)*G)) and synchronous step:          */
/*   R-phase: lanes needing a reset: s=reset(), a=get_action(s)              */
/*            (UCB: all read N,t; then N[s][a]+=1 per lane, t+=#calls)       */
/*   S-phase: (s2,r,term)=step(a); a2=get_action(s2) (same UCB snapshot rule) */
/*            train lanes: td from the Q snapshot; every entry moves by the   */
/*            MEAN of the contributions it received, at the end of the step. */
/* Every K=sync_every steps the groups merge: each entry takes the mean over  */
/* the groups that changed it; UCB N and t are summed.                       */
/*                                                                           */
/* Two representations of the shared Q (rlo_batch_q_repr):                   */
/*  FIXED40: int64 fixed point 2^-40, only where the range proof holds        */
/*           (o_delta_bound: one-step agent, single table, contracting       */
/*           bootstrap) — there |Q| never leaves max(|Q0|, R/(1-gamma)) and  */
/*           no clamp can engage.                                            */
/*  F64:     Q is f64 with the reference's full range (no clamp: entries      */
/*           that the reference drives to +-inf / NaN get there too,         */
/*           double_tabular_policy.rs:50-57).  A step's            */
/*           contributions d_i (f64, = lr*td or lr*(td*E)) to one entry are   */
/*           summed EXACTLY on the integer grid 2^e of the largest one        */
/*           (fq_step_combine): e = max(code(d_i), 1) - 1075 (code = biased   */
/*           exponent), so the largest is exact and the rest are rounded to   */
/*           its ulp; the sum is an int64 (order free, as on the GPU), the    */
/*           entry moves by ldexp(fl((double)sum * fl(1/n)), e).  n == 1 is   */
/*           exact: one lane reproduces Q[s][a] += lr*td                      */
/*           (tabular_policy.rs:35-38).  Any NaN / +-inf contribution makes   */
/*           the step's move NaN / +-inf (IEEE sum algebra).  Traces use one  */
/*           grid per group step, from the largest |td| and the trace bound. */
/*           The merge takes the mean of the changed groups' VALUES on the   */
/*           same kind of grid (plus headroom bits for many groups).  NaN is  */
/*           stored canonical (0x7FF8...), so equal states compare bitwise.  */
/* ======================================================================== */
typedef struct {
    rlo_rng rng;
    envstate st;
    uint32_t s, a;
    int need_reset, dflag, mode;
    double eps, epi_reward;
    uint64_t train_ep, eval_left, epi_len;
    double *trace;       /* [S][A] (traces agent) */
    uint32_t *vlist, vcnt; /* visited states in first-visit order */
    double *w;           /* NeuralPolicy parameters (private mode) */
    uint8_t *visited;
    /* private mode (G == 1): the lane is a whole reference agent */
    double *qd;          /* [P][S][A] f64 */
    uint64_t *n;         /* [S][A] (u128 in the reference) */
    uint64_t t;
    model_t model;       /* InternalModelAgent's RandomModel (private mode) */
} lane_t;

struct rlo_batch {
    rlo_config c;
    envdef E;
    uint32_t S, A, P, G, n_groups, K;
    int specials;        /* UCB + expected SARSA can produce inf/NaN */
    int priv;            /* G == 1: private f64 Q per lane, no merging */
    double *qd_g;        /* private mode: current lane's Q */
    int64_t *q_base;     /* [P][S][A] */
    uint8_t *f_base;
    uint64_t *n_base;    /* [S][A] UCB counts (u128 in the reference, upper_confidence_bound.rs:11) */
    uint64_t t_base;
    /* current group scratch */
    int64_t *q_g, *dq;
    uint32_t *dc;        /* contributions per entry this step */
    uint8_t *f_g, *df;
    uint64_t *n_g, *n_g_own;
    uint64_t t_g;
    /* merge accumulators */
    int64_t *acc_q, *acc_c; uint8_t *acc_f; int64_t *acc_n; int64_t acc_t;
    lane_t *lanes;
    uint64_t target_episodes, eval_at;
    int eval_only;
    int record;
    vec records;
    uint64_t stats[16];  /* rl_stats order; 8 = Q clamp hits, 9 = delta saturations */
    uint32_t plan;       /* Dyna planning steps per update (private mode only) */
    int reset_step;      /* reset-and-step schedule (shared mode, eps-greedy) */
    netdef net;          /* NeuralPolicy (private mode only) */
    double *feat, *w_g;  /* input features [S][in]; current lane's parameters */
    uint32_t net_gen;
    uint64_t last_done;  /* lanes DONE at the end of the last launch (rl_stats::done_lanes) */
    /* shared-Q representation (see the section header) */
    int qrepr;           /* RLO_QREPR_FIXED40 / RLO_QREPR_F64 */
    int q_forced;        /* rlo_batch_set_q_mode: 0 auto, 1 F64, 2 F64 with sequential sums */
    double q_abs0;       /* max |Q| at the last reset / set_q (the range proof's Q0) */
    double *qd_base, *qd_grp; /* F64: [P][S][A] merged base / the running group's copy (qd_g points at it) */
    uint32_t *ck; double *cd; size_t cn, ccap;   /* F64: this step's contributions (entry, d), lane order */
    uint32_t *fcode;     /* F64: per-entry max code of the step / merge */
    double *fseq;        /* F64 sequential variant: per-entry running sums */
    uint32_t td_code;    /* F64 traces: max code of the finite td of the group step */
    int trace_k;         /* F64 traces: 2^trace_k >= |lr| * (trace bound) * (1 + 2^-50) */
    uint64_t merge_groups;   /* learner groups over all ranks (merge grid headroom) */
    double *gvals;       /* F64 merge: every local group's Q after its launch [g][P][S][A] */
};

/* Fixed-point Q (shared mode).  |Q raw| <= 2^51, so every entry converts to
 * f64 exactly and (a+b)/2 of two entries is exact too: comparisons on raw
 * int64 values are then identical to the reference's f64 comparisons.
 * delta -> raw: NaN/inf become sticky flags; finite values are clamped to
 * +-2^51 and rounded half-to-even. */
#define Q_RAW_MAX ((int64_t)1 << 51)   /* |Q| <= 2048 */
#define D_RAW_MAX 0x1p51
static int64_t q_fix_sat(double d, uint8_t *flag, int *sat) {
    if (d != d) { *flag |= QF_NAN; return 0; }
    if (d == INFINITY) { *flag |= QF_PINF; return 0; }
    if (d == -INFINITY) { *flag |= QF_NINF; return 0; }
    double x = d * 0x1p40;
    if (sat && fabs(x) > D_RAW_MAX) *sat = 1;   /* rl_stats::delta_saturations */
    x = fmax(x, -D_RAW_MAX);
    x = fmin(x, D_RAW_MAX);
    return (int64_t)rint(x);
}
static inline int64_t q_clamp(int64_t v) {
    return v > Q_RAW_MAX ? Q_RAW_MAX : (v < -Q_RAW_MAX ? -Q_RAW_MAX : v);
}
/* the entry update with rl_stats::q_clamp_hits counted */
static inline int64_t q_clamp_count(rlo_batch *b, int64_t v) {
    if (v > Q_RAW_MAX || v < -Q_RAW_MAX) b->stats[8]++;
    return q_clamp(v);
}
static inline double q_val(int64_t raw, uint8_t fl) {
    if (fl) {
        if ((fl & QF_NAN) || ((fl & QF_PINF) && (fl & QF_NINF))) return NAN;
        return (fl & QF_PINF) ? INFINITY : -INFINITY;
    }
    return (double)raw * 0x1p-40;
}
static inline int64_t wrap_add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }

/* ---- F64 shared Q (section header above) ---- */
#define QNAN_BITS 0x7FF8000000000000ull
static inline uint64_t u_of(double x) { dbits b; b.d = x; return b.u; }
static inline double d_of(uint64_t u) { dbits b; b.u = u; return b.d; }
static inline double canon_nan(double x) { return x != x ? d_of(QNAN_BITS) : x; }
/* biased exponent field: 0 for zero / subnormal, 2047 for inf / NaN */
static inline uint32_t f64_code(double x) { return (uint32_t)(u_of(x) >> 52) & 0x7ffu; }
static inline uint8_t nf_flag(double x) { return x != x ? QF_NAN : (x > 0.0 ? QF_PINF : QF_NINF); }
/* the IEEE sum of contributions with these non-finite kinds */
static inline double nf_value(uint8_t f) {
    if ((f & QF_NAN) || ((f & QF_PINF) && (f & QF_NINF))) return d_of(QNAN_BITS);
    return (f & QF_PINF) ? INFINITY : -INFINITY;
}
/* d on the grid 2^e, rounded half-to-even (|result| < 2^53 when |d| < 2^(e+53)) */
static inline int64_t fq_raw(double d, int e) { return (int64_t)rint(ldexp(d, -e)); }
/* the mean of n grid values summing to `sum` */
static inline double fq_mean(int64_t sum, uint64_t n, int e) { return ldexp((double)sum * (1.0 / (double)n), e); }
static inline int fq_grid(uint32_t code) { return (int)(code > 1u ? code : 1u) - 1075; }
static int ceil_log2_u64(uint64_t n) {
    int h = 0;
    while (h < 64 && ((uint64_t)1 << h) < n) ++h;
    return h;
}
/* merge grid headroom: n values of < 2^(53-h) grid units stay below 2^63 for
 * up to 2^(10+h) groups (rlamd rl_host.cpp merge_headroom) */
static int fq_merge_headroom(uint64_t groups) {
    const int h = ceil_log2_u64(groups) - 10;
    return h > 0 ? h : 0;
}
/* traces grid: every contribution fl(lr * fl(td * E)) of a group step is below
 * 2^(max(code(td),1) - 1024 + k) with 2^k >= 4 * |lr| * Ebound * (1 + 2^-50) —
 * below 2^51 units of its grid, two guard bits that let the device convert a
 * contribution with the 1.5*2^52 magic add — where
 * Ebound bounds an accumulating trace (elegibility_traces_agent.rs:75-96: E += 1
 * on a visit, E *= gamma*lambda after each sweep): 1/(1-|gl|) for |gl| < 1, else
 * the geometric sum over the longest episode.  Same formula as the product's
 * host (rl_host.cpp trace_grid_k). */
int rlo_trace_grid_k(double lr, double gamma, double lambda_, uint32_t max_steps, int32_t env) {
    const double gl = gamma * lambda_, a = fabs(gl);
    double eb;
    if (a < 1.0) {
        eb = 1.0 / (1.0 - a);
    } else {
        /* sum_{k=0..T} a^k in closed form (T in 64 bits: max_steps + 1 cannot wrap;
         * O(1)); expm1/log1p keep it accurate for a just above 1,
         * and it is +inf when the sum overflows */
        const uint64_t T = env == RLO_ENV_BLACKJACK ? 32u : (uint64_t)max_steps + 1u;
        eb = a == 1.0 ? (double)(T + 1u) : expm1((double)(T + 1u) * log1p(a - 1.0)) / (a - 1.0);
    }
    const double x = fabs(lr) * eb * (1.0 + 0x1p-50) * 1.0001;
    if (!(x > 0.0)) return 0;
    if (!(x < INFINITY)) return 1100;
    int ex;
    (void)frexp(x, &ex);
    ex += 2;   /* two guard bits: |raw| < 2^51 */
    return ex < -1100 ? -1100 : (ex > 1100 ? 1100 : ex);
}
/* a value the fixed point holds exactly and in range */
static inline int fix_exact(double v) {
    if (!(fabs(v) <= 2048.0)) return 0;
    const double x = v * 0x1p40;
    return x == rint(x);
}

/* ---- the range proof that admits the fixed point (rlamd rl_host.cpp delta_bound,
 * same conditions): the one-step agent on a single table, with a bootstrap that
 * is a sub-convex combination of Q values (SARSA's pick, Q-learning's max,
 * expected SARSA over eps-greedy), keeps every entry within
 * max(|Q0|, R/(1-gamma)); the double policy (double_tabular_policy.rs:50-57,
 * A - B grows by (1 + lr) per update pair), eligibility traces and UCB +
 * expected SARSA (u_i / sum(u) weights) are not contractions. */
static double o_reward_bound(int env) {
    switch (env) {
    case RLO_ENV_FROZEN_LAKE: return 1.0;
    case RLO_ENV_FROZEN_LAKE_EDITED: return 10.0;
    case RLO_ENV_CLIFF_WALKING: return 100.0;
    case RLO_ENV_TAXI: return 20.0;
    case RLO_ENV_BLACKJACK: return 1.0;
    default: return INFINITY;
    }
}
static double o_delta_bound(const rlo_batch *b) {
    const rlo_config *c = &b->c;
    if (b->priv || b->feat) return INFINITY;
    if (c->agent != RLO_AGENT_ONE_STEP || c->policy != RLO_POLICY_TABULAR) return INFINITY;
    if (c->selector == RLO_SEL_UCB && c->algo == RLO_ALGO_EXPECTED_SARSA) return INFINITY;
    const double lr = c->lr, g = c->gamma;
    if (!(lr >= 0.0 && g >= 0.0 && g < 1.0 && isfinite(b->q_abs0))) return INFINITY;
    if (!(lr <= 1.0)) return INFINITY;
    if (c->selector == RLO_SEL_EPS_GREEDY && c->algo == RLO_ALGO_EXPECTED_SARSA) {
        const int dec = c->decay_kind == RLO_DECAY_MUL ? (c->eps_decay >= 0.0 && c->eps_decay <= 1.0)
                                                       : c->eps_decay >= 0.0;
        if (!(c->eps0 >= 0.0 && c->eps0 <= 1.0 && c->eps_final >= 0.0 && dec)) return INFINITY;
    }
    const double R = o_reward_bound(c->env);
    const double mb = b->q_abs0 > R / (1.0 - g) ? b->q_abs0 : R / (1.0 - g);
    if (!(mb <= 2000.0)) return INFINITY;
    const double ep_len = c->env == RLO_ENV_BLACKJACK ? 1.0 : (double)c->max_steps + 1.0;
    if (!(ep_len * R * 65536.0 < 0x1p50)) return INFINITY;
    return lr * (R + (1.0 + g) * mb);
}
/* slippery FrozenLake tables stay f64 under "auto": the fixed point's rounding
 * flips greedy ties, trajectories part and Q leaves the 1e-5 bar (rl_host.cpp
 * fix_faithful; tests/golden/longrun.json repr_drift_curve) */
static int o_faithful(const rlo_batch *b) {
    return !((b->c.env == RLO_ENV_FROZEN_LAKE || b->c.env == RLO_ENV_FROZEN_LAKE_EDITED) && b->c.slippery);
}
static int o_proven(const rlo_batch *b) {
    return o_delta_bound(b) < 2000.0 && (b->q_forced == RLO_QMODE_FIXED_RANGE || o_faithful(b));
}

/* representation changes: fixed point -> f64 is exact (|raw| <= 2^51) */
static void o_to_f64(rlo_batch *b) {
    const size_t nq = (size_t)b->P * b->S * b->A;
    for (size_t k = 0; k < nq; ++k) b->qd_base[k] = q_val(b->q_base[k], b->f_base[k]);
    b->qrepr = RLO_QREPR_F64;
}
/* qd_base holds a freshly set table: the fixed point when it is allowed and exact */
static void o_choose_repr(rlo_batch *b) {
    const size_t nq = (size_t)b->P * b->S * b->A;
    b->qrepr = RLO_QREPR_F64;
    if (b->priv || (b->q_forced && b->q_forced != RLO_QMODE_FIXED_RANGE) || !o_proven(b)) return;
    for (size_t k = 0; k < nq; ++k)
        if (!fix_exact(b->qd_base[k])) return;
    for (size_t k = 0; k < nq; ++k) { b->q_base[k] = (int64_t)(b->qd_base[k] * 0x1p40); b->f_base[k] = 0; }
    b->qrepr = RLO_QREPR_FIXED40;
}
static void o_set_abs0(rlo_batch *b, const double *v, size_t n) {
    b->q_abs0 = 0.0;
    for (size_t k = 0; k < n; ++k) {
        const double a = fabs(v[k]);
        b->q_abs0 = a != a ? INFINITY : (a > b->q_abs0 ? a : b->q_abs0);
    }
}
/* after a selector / algorithm change: a fixed-point table whose proof no longer holds goes f64 */
static void o_recheck_repr(rlo_batch *b) {
    if (!b->priv && b->qrepr == RLO_QREPR_FIXED40 && !o_proven(b)) o_to_f64(b);
}

static void b_row(const rlo_batch *b, uint32_t tbl, uint32_t s, double *out) {
    size_t base = ((size_t)tbl * b->S + s) * b->A;
    if (b->feat) {                    /* NeuralPolicy::get_values / predict (neural_policy.rs:43-53) */
        double opre[MAXA];
        net_forward(&b->net, b->w_g, b->feat + (size_t)s * b->net.in, opre, out);
        return;
    }
    if (b->priv || b->qrepr == RLO_QREPR_F64) {
        for (uint32_t i = 0; i < b->A; ++i) out[i] = b->qd_g[base + i];
        return;
    }
    for (uint32_t i = 0; i < b->A; ++i) out[i] = q_val(b->q_g[base + i], b->f_g[base + i]);
}
static void b_predict(const rlo_batch *b, uint32_t s, double *out) {
    b_row(b, 0, s, out);
    if (b->P == 2) {
        double o2[MAXA];
        b_row(b, 1, s, o2);
        for (uint32_t i = 0; i < b->A; ++i) out[i] = (out[i] + o2[i]) / 2.0;
    }
}
/* get_action against the group snapshot; UCB increments are returned, not applied */
static uint32_t b_select(rlo_batch *b, lane_t *L, uint32_t s) {
    double v[MAXA];
    b_predict(b, s, v);
    if (b->c.selector == RLO_SEL_EPS_GREEDY) {
        if (L->eps != 0.0 && eps_test(&L->rng, L->eps)) return uniform_action(&L->rng, b->A);
        return argmax_d(v, b->A);
    }
    const uint64_t *n = &b->n_g[(size_t)s * b->A];
    double lnt = rlo_log((double)b->t_g);
    double u[MAXA];
    for (uint32_t i = 0; i < b->A; ++i) u[i] = ucb_value(v[i], b->c.ucb_c, lnt, (double)n[i]);
    return argmax_d(u, b->A);
}

static void lane_init(rlo_batch *b, lane_t *L, uint64_t gid) {
    memset(&L->st, 0, sizeof L->st);
    rng_seed(&L->rng, b->c.seed, gid);
    if (b->c.env == RLO_ENV_BLACKJACK) bj_initialize_hands(&L->st, &L->rng);
    L->need_reset = 1; L->dflag = 1; L->mode = RLO_MODE_TRAIN;
    L->eps = b->c.eps0;
    L->train_ep = L->eval_left = L->epi_len = 0;
    L->epi_reward = 0.0;
    L->s = L->a = 0;
}

rlo_batch *rlo_batch_create(const rlo_config *c) {
    rlo_batch *b = (rlo_batch *)calloc(1, sizeof(rlo_batch));
    b->c = *c;
    if (build_env(&b->E, c) || c->n_lanes == 0 || c->group_size == 0 || c->sync_every == 0) {
        free(b);
        return NULL;
    }
    b->S = b->E.S; b->A = b->E.A; b->P = c->policy == RLO_POLICY_DOUBLE ? 2 : 1;
    b->G = c->group_size; b->K = c->sync_every;
    b->n_groups = (c->n_lanes + b->G - 1) / b->G;
    b->specials = c->selector == RLO_SEL_UCB && c->algo == RLO_ALGO_EXPECTED_SARSA;
    b->priv = b->G == 1;
    if (b->G > 1024) { free(b); return NULL; }
    if (c->policy == RLO_POLICY_NEURAL) {
        if (!b->priv || net_make(c, b->A, &b->net)) { free(b); return NULL; }
        b->feat = (double *)malloc(sizeof(double) * b->S * b->net.in);
        net_features(&b->E, &b->net, c->net_input, b->feat);
    }
    size_t nq = (size_t)b->P * b->S * b->A, nsa = (size_t)b->S * b->A;
    b->q_base = (int64_t *)malloc(nq * 8); b->f_base = (uint8_t *)calloc(nq, 1);
    b->q_g = (int64_t *)malloc(nq * 8); b->f_g = (uint8_t *)calloc(nq, 1);
    b->dq = (int64_t *)calloc(nq, 8); b->df = (uint8_t *)calloc(nq, 1);
    b->dc = (uint32_t *)calloc(nq, 4);
    b->acc_q = (int64_t *)calloc(nq, 8); b->acc_f = (uint8_t *)calloc(nq, 1);
    b->acc_c = (int64_t *)calloc(nq, 8);
    b->n_base = (uint64_t *)calloc(nsa, 8); b->n_g = b->n_g_own = (uint64_t *)calloc(nsa, 8);
    b->acc_n = (int64_t *)calloc(nsa, 8);
    b->qd_base = (double *)calloc(nq, 8); b->qd_grp = (double *)calloc(nq, 8);
    b->fcode = (uint32_t *)calloc(nq, 4); b->fseq = (double *)calloc(nq, 8);
    b->merge_groups = b->n_groups;
    b->trace_k = rlo_trace_grid_k(c->lr, c->gamma, c->lambda_, c->max_steps, c->env);
    b->records.esz = sizeof(rlo_record);
    b->lanes = (lane_t *)calloc(c->n_lanes, sizeof(lane_t));
    for (uint32_t i = 0; i < c->n_lanes; ++i) {
        if (c->agent == RLO_AGENT_TRACES) {
            b->lanes[i].trace = (double *)calloc(nsa, sizeof(double));
            b->lanes[i].visited = (uint8_t *)calloc(b->S, 1);
            b->lanes[i].vlist = (uint32_t *)calloc(b->S, sizeof(uint32_t));
        }
        if (b->feat) b->lanes[i].w = (double *)malloc(sizeof(double) * b->net.np);
        if (b->priv) {
            b->lanes[i].qd = (double *)malloc(nq * sizeof(double));
            b->lanes[i].n = (uint64_t *)calloc(nsa, sizeof(uint64_t));
        }
        lane_init(b, &b->lanes[i], c->lane_offset + i);
    }
    b->net_gen = (uint32_t)-1;           /* the first reset is NeuralPolicy::new (generation 0) */
    rlo_batch_reset(b);
    return b;
}
void rlo_batch_destroy(rlo_batch *b) {
    if (!b) return;
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
        free(b->lanes[i].trace); free(b->lanes[i].visited); free(b->lanes[i].qd); free(b->lanes[i].n);
        free(b->lanes[i].vlist); free(b->lanes[i].w);
        model_free(&b->lanes[i].model);
    }
    free(b->lanes); free(b->q_base); free(b->f_base); free(b->q_g); free(b->f_g); free(b->dq);
    free(b->df); free(b->dc); free(b->acc_c); free(b->acc_q); free(b->acc_f); free(b->n_base); free(b->n_g_own); free(b->acc_n);
    free(b->records.p); free(b->feat);
    free(b->qd_base); free(b->qd_grp); free(b->fcode); free(b->fseq); free(b->ck); free(b->cd); free(b->gvals);
    free(b);
}
/* Agent::reset: policy cleared to the default row, selector state fresh, lane
 * ε restored; env/RNG/double-flag untouched (one_step_agent.rs:43-46,
 * double_tabular_policy.rs:62-65 keeps policy_flag). */
void rlo_batch_reset(rlo_batch *b) {
    size_t nq = (size_t)b->P * b->S * b->A;
    for (size_t i = 0; i < nq; ++i) b->qd_base[i] = canon_nan(b->c.q_default);
    o_set_abs0(b, &b->c.q_default, 1);
    o_choose_repr(b);
    memset(b->n_base, 0, sizeof(uint64_t) * b->S * b->A);
    b->t_base = 1;
    b->net_gen++;
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
        lane_t *L = &b->lanes[i];
        L->eps = b->c.eps0;
        if (L->w) net_init(&b->net, L->w, b->c.seed, b->c.lane_offset + i, b->net_gen);  /* Network::reset */
        if (b->priv) {
            for (size_t k = 0; k < nq; ++k) L->qd[k] = b->c.q_default;
            memset(L->n, 0, sizeof(uint64_t) * b->S * b->A);
            L->t = 1;
        }
        L->model.cnt = 0;                    /* model.reset (internal_model_agent.rs:79-82) */
    }
}
void rlo_batch_set_reset_step(rlo_batch *b, int on) { b->reset_step = on != 0; }
int rlo_batch_set_planning(rlo_batch *b, uint32_t planning_steps) {
    if (planning_steps && !b->priv) return -1;   /* Dyna: private agents only */
    b->plan = planning_steps;
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
        model_free(&b->lanes[i].model);
        if (planning_steps) model_alloc(&b->lanes[i].model, (size_t)b->S * b->A);
    }
    return 0;
}
void rlo_batch_set_selector(rlo_batch *b, int32_t sel) {
    b->c.selector = sel;
    b->specials = b->c.selector == RLO_SEL_UCB && b->c.algo == RLO_ALGO_EXPECTED_SARSA;
    o_recheck_repr(b);
    memset(b->n_base, 0, sizeof(uint64_t) * b->S * b->A);
    b->t_base = 1;
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
        b->lanes[i].eps = b->c.eps0;
        if (b->priv) { memset(b->lanes[i].n, 0, sizeof(uint64_t) * b->S * b->A); b->lanes[i].t = 1; }
    }
}
void rlo_batch_set_algo(rlo_batch *b, int32_t algo) {
    b->c.algo = algo;
    b->specials = b->c.selector == RLO_SEL_UCB && b->c.algo == RLO_ALGO_EXPECTED_SARSA;
    o_recheck_repr(b);
}
/* RLO_QMODE_AUTO: the fixed point where the range proof holds (and the table is
 * exact in it), else f64; RLO_QMODE_F64: f64 always; RLO_QMODE_F64_SEQ (oracle
 * only): f64 with every step / merge sum formed sequentially in lane / group
 * order instead of on the exponent grid — the drift reference; RLO_QMODE_FIXED_RANGE
 * (oracle only): the fixed point wherever the range proof holds, slippery maps
 * included (round 5's "auto": the repr_drift_curve measurement) */
void rlo_batch_set_q_mode(rlo_batch *b, int mode) {
    if (b->priv) return;
    b->q_forced = mode;
    if (mode != RLO_QMODE_AUTO && mode != RLO_QMODE_FIXED_RANGE) {
        if (b->qrepr == RLO_QREPR_FIXED40) o_to_f64(b);
        return;
    }
    if (b->qrepr == RLO_QREPR_F64) {
        const size_t nq = (size_t)b->P * b->S * b->A;
        const double keep = b->q_abs0;
        o_set_abs0(b, b->qd_base, nq);
        o_choose_repr(b);
        if (b->qrepr == RLO_QREPR_F64) b->q_abs0 = keep;
    }
}
int rlo_batch_q_repr(const rlo_batch *b) { return b->priv ? RLO_QREPR_PRIVATE : b->qrepr; }
void rlo_batch_set_merge_groups(rlo_batch *b, uint64_t total_groups) {
    b->merge_groups = total_groups ? total_groups : b->n_groups;
}
void rlo_batch_set_record(rlo_batch *b, int e) { b->record = e; }

static void add_delta(rlo_batch *b, uint32_t tbl, uint32_t s, uint32_t a, double delta) {
    size_t k = ((size_t)tbl * b->S + s) * b->A + a;
    if (b->priv) {                   /* Q[s][a] += lr*td exactly as tabular_policy.rs:36 */
        b->qd_g[k] += delta;
        return;
    }
    if (b->qrepr == RLO_QREPR_F64) {   /* combined at the end of the step (fq_step_combine) */
        if (b->cn == b->ccap) {
            b->ccap = b->ccap ? 2 * b->ccap : 4096;
            b->ck = (uint32_t *)realloc(b->ck, b->ccap * sizeof(uint32_t));
            b->cd = (double *)realloc(b->cd, b->ccap * sizeof(double));
        }
        b->ck[b->cn] = (uint32_t)k;
        b->cd[b->cn] = delta;
        b->cn++;
        return;
    }
    uint8_t fl = 0;
    int sat = 0;
    int64_t d = q_fix_sat(delta, &fl, &sat);
    b->stats[9] += (uint64_t)sat;
    b->dq[k] = wrap_add(b->dq[k], d);
    b->dc[k] += 1;
    b->df[k] |= fl;
}

/* The shared-mode combination rule: an entry moves by the MEAN of the n
 * contributions it received (this step's lanes, or the groups that changed it
 * at a merge): trunc((double)sum * (1.0/n)), with 1.0/n correctly rounded.
 * n == 1 is exact (|sum| <= 2^53, so one lane reproduces the reference update);
 * n == 0 has sum == 0.  Conversions, the reciprocal and the product are
 * correctly rounded IEEE operations, so host and gfx950 agree bit for bit (the
 * device reads 1.0/n from a table, rlamd rl_train_impl.h mean_delta). */
static int64_t mean_delta(int64_t sum, int64_t n) {
    if (n <= 0) return 0;
    return (int64_t)trunc((double)sum * (1.0 / (double)n));
}

/* F64: the end of a group step.  Per entry, the step's contributions (lane
 * order in cd[]) are combined order-free: largest code -> grid 2^e, integer sum,
 * mean; non-finite contributions give the IEEE result.  RLO_QMODE_F64_SEQ sums
 * the f64 contributions in lane order instead (the drift reference). */
static void fq_step_combine(rlo_batch *b) {
    const size_t nq = (size_t)b->P * b->S * b->A;
    const int traces = b->c.agent == RLO_AGENT_TRACES;
    const int seq = b->q_forced == RLO_QMODE_F64_SEQ;
    memset(b->dq, 0, nq * 8);
    memset(b->dc, 0, nq * 4);
    memset(b->df, 0, nq);
    memset(b->fcode, 0, nq * 4);
    memset(b->fseq, 0, nq * 8);
    for (size_t i = 0; i < b->cn; ++i) {
        const uint32_t k = b->ck[i];
        const double d = b->cd[i];
        b->dc[k]++;
        if (!isfinite(d)) b->df[k] |= nf_flag(d);
        else if (f64_code(d) > b->fcode[k]) b->fcode[k] = f64_code(d);
    }
    /* traces: one grid for the group step (the contributions of a row come from
     * many lanes' sweeps; the bound is known before any is formed) */
    const int e_tr = fq_grid(b->td_code) + b->trace_k;
    for (size_t i = 0; i < b->cn; ++i) {
        const uint32_t k = b->ck[i];
        const double d = b->cd[i];
        if (!isfinite(d)) continue;
        b->dq[k] += fq_raw(d, traces ? e_tr : fq_grid(b->fcode[k]));
        b->fseq[k] += d;
    }
    for (size_t k = 0; k < nq; ++k) {
        if (!b->dc[k]) continue;
        double mv;
        if (b->df[k]) mv = nf_value(b->df[k]);
        else if (seq) mv = b->fseq[k] * (1.0 / (double)b->dc[k]);
        else mv = fq_mean(b->dq[k], b->dc[k], traces ? e_tr : fq_grid(b->fcode[k]));
        b->qd_g[k] = canon_nan(b->qd_g[k] + mv);
    }
    b->cn = 0;
    b->td_code = 0;
}

/* Policy::update with x = td (one-step) or td * E[o][b] (traces):
 * tabular Q[s][a] += lr * x; neural y = get_values(s), y[a] += x, fit */
static void b_policy_update(rlo_batch *b, uint32_t tbl, uint32_t s, uint32_t a, double x) {
    if (b->feat) {
        double y[MAXA], opre[MAXA];
        const double *in = b->feat + (size_t)s * b->net.in;
        net_forward(&b->net, b->w_g, in, opre, y);
        y[a] += x;
        net_fit(&b->net, b->w_g, in, y, b->c.lr);
        return;
    }
    add_delta(b, tbl, s, a, b->c.lr * x);
}

/* Agent::update of one lane against the current Q / UCB state
 * (one_step_agent.rs:53-86, elegibility_traces_agent.rs:61-104), with
 * after_update and the termination hooks */
static double b_update(rlo_batch *b, lane_t *L, uint32_t s, uint32_t a, double r, int term, uint32_t s2,
                       uint32_t a2) {
    const uint32_t A = b->A;
    const int ucb = b->c.selector == RLO_SEL_UCB;
    uint32_t vt = (b->P == 2 && !L->dflag) ? 1 : 0;   /* get_values table */
    uint32_t ut = (b->P == 2 && L->dflag) ? 1 : 0;    /* update table */
    double q2[MAXA], p[MAXA], q[MAXA];
    b_row(b, vt, s2, q2);
    if (!ucb) eps_probs(L->eps, q2, A, p);
    else if (b->c.algo == RLO_ALGO_EXPECTED_SARSA) {
        uint64_t n64[MAXA];
        for (uint32_t i = 0; i < A; ++i) n64[i] = b->n_g[(size_t)s2 * A + i];
        ucb_probs(q2, n64, b->t_g, b->c.ucb_c, A, p);
    }
    double fq = future_q(b->c.algo, q2, a2, p, A);
    b_row(b, vt, s, q);
    double td = r + b->c.gamma * fq - q[a];
    if (b->c.agent == RLO_AGENT_ONE_STEP) {
        b_policy_update(b, ut, s, a, td);
    } else {
        /* F64 traces: the group step's grid follows its largest finite |td| */
        if (!b->priv && b->qrepr == RLO_QREPR_F64 && isfinite(td) && f64_code(td) > b->td_code)
            b->td_code = f64_code(td);
        L->trace[(size_t)s * A + a] += 1.0;
        if (!L->visited[s]) { L->visited[s] = 1; L->vlist[L->vcnt++] = s; }
        for (uint32_t vi = 0; vi < L->vcnt; ++vi) {   /* first-visit order (see f_update) */
            const uint32_t o = L->vlist[vi];
            b->stats[7]++;                    /* visited-set entries swept (V per step) */
            for (uint32_t bb = 0; bb < A; ++bb) {
                double *e = &L->trace[(size_t)o * A + bb];
                b_policy_update(b, ut, o, bb, td * *e);
                *e *= b->c.gamma * b->c.lambda_;
            }
        }
    }
    if (b->P == 2) L->dflag = !L->dflag;
    if (term) {
        if (b->c.agent == RLO_AGENT_TRACES) {
            memset(L->trace, 0, sizeof(double) * b->S * A);
            memset(L->visited, 0, b->S);
            L->vcnt = 0;
        }
        if (!ucb) L->eps = decay_eps(&b->c, L->eps);
    }
    return td;
}

/* One synchronous step of a learner group.  Every live lane does exactly one
 * of (src/agent.rs:83-106 cut at its get_action calls):
 *   RESET: s = env.reset(); a = get_action(s)                 (:83-84)
 *   STEP:  (s',r,term) = env.step(a); a' = get_action(s'); update  (:88-101)
 * All lanes read the step-start snapshot (Q, UCB N/t); UCB increments are
 * applied after every selection; Q moves by the mean of the step's deltas.
 * For one lane this is the reference's sequence exactly. */
static void group_step(rlo_batch *b, uint32_t lane0, uint32_t nl, rlo_record *rec) {
    const uint32_t A = b->A;
    const int ucb = b->c.selector == RLO_SEL_UCB;
    uint32_t s2v[1024], a2v[1024], kind[1024];
    double rv[1024];
    int tv[1024];
    uint32_t nsel = 0;
    /* ---- env + selection against the snapshot ---- */
    for (uint32_t j = 0; j < nl; ++j) {
        lane_t *L = &b->lanes[lane0 + j];
        kind[j] = 0;
        if (L->mode == RLO_MODE_DONE) continue;
        if (L->need_reset && b->reset_step && !b->priv && !ucb) {
            /* reset-and-step schedule: env.reset() + get_action against the
             * snapshot, then the step from (s0, a0) (src/agent.rs:83-89) */
            kind[j] = 3;
            L->s = env_reset(&b->E, &L->st, &L->rng);
            L->a = b_select(b, L, L->s);
            L->need_reset = 0; L->epi_reward = 0.0; L->epi_len = 0;
            if (env_step(&b->E, &L->st, L->a, &L->rng, &s2v[j], &rv[j], &tv[j])) abort();
        } else if (L->need_reset) {
            kind[j] = 1;
            s2v[j] = env_reset(&b->E, &L->st, &L->rng);
            rv[j] = 0.0; tv[j] = 0;
        } else {
            kind[j] = 2;
            if (env_step(&b->E, &L->st, L->a, &L->rng, &s2v[j], &rv[j], &tv[j])) abort();
        }
        a2v[j] = b_select(b, L, s2v[j]);
        nsel++;
    }
    if (ucb) {
        for (uint32_t j = 0; j < nl; ++j)
            if (kind[j]) b->n_g[(size_t)s2v[j] * A + a2v[j]] += 1;
        b->t_g += nsel;
    }
    /* ---- TD update of the STEP lanes against the Q snapshot ---- */
    size_t nq = (size_t)b->P * b->S * A;
    memset(b->dq, 0, nq * 8);
    memset(b->dc, 0, nq * 4);
    memset(b->df, 0, nq);
    b->cn = 0;
    b->td_code = 0;
    for (uint32_t j = 0; j < nl; ++j) {
        lane_t *L = &b->lanes[lane0 + j];
        rlo_record *R = rec ? &rec[j] : NULL;
        if (R) { memset(R, 0, sizeof *R); R->mode = (uint8_t)L->mode; R->kind = (uint8_t)kind[j]; }
        if (kind[j] == 0) continue;
        if (kind[j] == 1) {                   /* RESET: new episode, first action */
            L->s = s2v[j]; L->a = a2v[j];
            L->need_reset = 0; L->epi_reward = 0.0; L->epi_len = 0;
            if (R) { R->s = L->s; R->a = (uint8_t)L->a; }
            continue;
        }
        uint32_t s = L->s, a = L->a, s2 = s2v[j], a2 = a2v[j];
        double r = rv[j];
        int term = tv[j];
        double td = 0.0;
        if (L->mode == RLO_MODE_TRAIN) {
            td = b_update(b, L, s, a, r, term, s2, a2);
            if (b->plan) {                        /* InternalModelAgent (private mode) */
                model_add(&L->model, s * A + a, s2, r);
                for (uint32_t i = 0; i < b->plan; ++i) {
                    uint32_t jj = gen_index(&L->rng, L->model.cnt);
                    uint32_t k = L->model.key[jj], ps = k / A, pa = k % A, ps2 = L->model.s2[jj];
                    double pr = L->model.r[jj];
                    uint32_t na = b_select(b, L, ps2);
                    if (ucb) { b->n_g[(size_t)ps2 * A + na] += 1; b->t_g += 1; }
                    b_update(b, L, ps, pa, pr, 0, ps2, na);
                }
            }
            b->stats[0]++;
        } else {
            b->stats[1]++;
        }
        if (R) {
            R->s = s; R->a = (uint8_t)a; R->s2 = s2; R->a2 = (uint8_t)a2;
            R->r = r; R->term = (uint8_t)term; R->td = td;
        }
        /* bookkeeping: src/agent.rs:98-116 */
        L->epi_reward += r;
        L->epi_len++;
        L->s = s2; L->a = a2;
        if (term) {
            L->need_reset = 1;
            if (L->mode == RLO_MODE_TRAIN) {
                uint64_t ep = L->train_ep++;
                b->stats[2]++;
                b->stats[4] += (uint64_t)(int64_t)rint(L->epi_reward * 65536.0);
                if (b->eval_at && ep % b->eval_at == 0) {
                    L->mode = RLO_MODE_EVAL;
                    L->eval_left = b->c.eval_episodes;
                    if (L->eval_left == 0) L->mode = RLO_MODE_TRAIN;
                }
                if (L->mode == RLO_MODE_TRAIN && b->target_episodes && L->train_ep >= b->target_episodes)
                    L->mode = RLO_MODE_DONE;
            } else {
                b->stats[3]++;
                if (--L->eval_left == 0) {
                    int fin = b->eval_only || (b->target_episodes && L->train_ep >= b->target_episodes);
                    L->mode = fin ? RLO_MODE_DONE : RLO_MODE_TRAIN;
                }
            }
        }
    }
    if (b->priv) return;
    if (b->qrepr == RLO_QREPR_F64) {
        fq_step_combine(b);
        return;
    }
    for (size_t k = 0; k < nq; ++k) {
        b->q_g[k] = q_clamp_count(b, b->q_g[k] + mean_delta(b->dq[k], b->dc[k]));
        b->f_g[k] |= b->df[k];
    }
}

/* Merge buffer, same layout as the GPU's (rl_kparams.h): PSA "max" words
 * [PSA codes] then the "sum" words [PSA sums][PSA group counts][SA dN][1 dt]
 * [3*PSA flag counts] (int64).  Multi-rank (every rank runs its groups):
 *   launch_groups -> all-reduce MAX of the max words -> fold -> all-reduce SUM of
 *   the sum words -> apply_delta
 * Every rank then applies the identical total.  The fixed point uses only the
 * sum words (integer sums of the groups' changes; fold is a no-op). */
uint64_t rlo_batch_delta_words(const rlo_batch *b) {
    const size_t nq = (size_t)b->P * b->S * b->A, nsa = (size_t)b->S * b->A;
    return nq + 2 * nq + nsa + 1 + 3 * nq;
}
uint64_t rlo_batch_delta_max_words(const rlo_batch *b) { return (uint64_t)b->P * b->S * b->A; }

/* run every local group for K synchronous steps and ADD its changes to delta
 * (shared mode); private mode just runs the lanes (delta untouched) */
void rlo_batch_launch_groups(rlo_batch *b, int64_t *delta) {
    size_t nq = (size_t)b->P * b->S * b->A, nsa = (size_t)b->S * b->A;
    rlo_record *tmp = b->record ? (rlo_record *)malloc(sizeof(rlo_record) * b->G) : NULL;
    size_t rec0 = b->records.n;
    if (b->record) {
        rlo_record z;
        memset(&z, 0, sizeof z);
        for (size_t i = 0; i < (size_t)b->K * b->c.n_lanes; ++i) vpush(&b->records, &z);
    }
    if (b->priv) {
        for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
            lane_t *L = &b->lanes[i];
            b->qd_g = L->qd; b->n_g = L->n; b->t_g = L->t; b->w_g = L->w;
            for (uint32_t k = 0; k < b->K; ++k) {
                group_step(b, i, 1, tmp);
                if (tmp) ((rlo_record *)b->records.p)[rec0 + (size_t)k * b->c.n_lanes + i] = tmp[0];
            }
            L->t = b->t_g;
        }
        b->n_g = b->n_g_own;
        free(tmp);
        return;
    }
    int64_t *dmax = delta;
    int64_t *dsum = delta + nq, *dcnt = dsum + nq, *dn = dsum + 2 * nq, *dt = dn + nsa, *fc = dt + 1;
    const int f64 = b->qrepr == RLO_QREPR_F64;
    if (f64 && !b->gvals) b->gvals = (double *)malloc(sizeof(double) * nq * b->n_groups);
    for (uint32_t g = 0; g < b->n_groups; ++g) {
        uint32_t lane0 = g * b->G;
        uint32_t nl = b->c.n_lanes - lane0 < b->G ? b->c.n_lanes - lane0 : b->G;
        if (f64) { b->qd_g = b->qd_grp; memcpy(b->qd_g, b->qd_base, nq * 8); }
        else { memcpy(b->q_g, b->q_base, nq * 8); memcpy(b->f_g, b->f_base, nq); }
        memcpy(b->n_g, b->n_base, nsa * 8); b->t_g = b->t_base;
        for (uint32_t k = 0; k < b->K; ++k) {
            group_step(b, lane0, nl, tmp);
            if (tmp) {
                rlo_record *dst = (rlo_record *)b->records.p + rec0 + (size_t)k * b->c.n_lanes + lane0;
                memcpy(dst, tmp, sizeof(rlo_record) * nl);
            }
        }
        if (f64) {   /* the group's values stay for the fold; max code / count / kinds now */
            memcpy(b->gvals + (size_t)g * nq, b->qd_g, nq * 8);
            for (size_t i = 0; i < nq; ++i) {
                const double v = b->qd_g[i];
                if (u_of(v) == u_of(b->qd_base[i])) continue;
                dcnt[i] += 1;
                if (!isfinite(v)) {
                    const uint8_t f = nf_flag(v);
                    fc[(f == QF_NAN ? 0 : f == QF_PINF ? 1 : 2) * nq + i] += 1;
                } else if ((int64_t)f64_code(v) > dmax[i]) {
                    dmax[i] = f64_code(v);
                }
            }
        } else {
            for (size_t i = 0; i < nq; ++i) {
                const int64_t d = (int64_t)((uint64_t)b->q_g[i] - (uint64_t)b->q_base[i]);
                if (d) { dsum[i] = wrap_add(dsum[i], d); dcnt[i] += 1; }
                const uint8_t nf = (uint8_t)(b->f_g[i] & ~b->f_base[i]);
                if (nf & QF_NAN) fc[i] += 1;
                if (nf & QF_PINF) fc[nq + i] += 1;
                if (nf & QF_NINF) fc[2 * nq + i] += 1;
            }
        }
        for (size_t i = 0; i < nsa; ++i) dn[i] += (int64_t)(b->n_g[i] - b->n_base[i]);
        *dt += (int64_t)(b->t_g - b->t_base);
    }
    free(tmp);
}

/* F64 merge, second phase: the local groups' changed finite values on the grid
 * of the (all-reduced) max code, + headroom bits for the number of groups */
void rlo_batch_fold(rlo_batch *b, int64_t *delta) {
    if (b->priv || b->qrepr != RLO_QREPR_F64) return;
    const size_t nq = (size_t)b->P * b->S * b->A;
    const int64_t *dmax = delta;
    int64_t *dsum = delta + nq;
    const int hb = fq_merge_headroom(b->merge_groups);
    memset(b->fseq, 0, nq * 8);
    for (uint32_t g = 0; g < b->n_groups; ++g) {
        const double *gv = b->gvals + (size_t)g * nq;
        for (size_t i = 0; i < nq; ++i) {
            const double v = gv[i];
            if (u_of(v) == u_of(b->qd_base[i]) || !isfinite(v)) continue;
            dsum[i] += fq_raw(v, fq_grid((uint32_t)dmax[i]) + hb);
            b->fseq[i] += v;
        }
    }
}

/* every entry that some group changed takes the mean over those groups
 * (fixed point: Q_base += mean of the changes; f64: the mean of the values);
 * UCB counters summed */
void rlo_batch_apply_delta(rlo_batch *b, const int64_t *delta) {
    size_t nq = (size_t)b->P * b->S * b->A, nsa = (size_t)b->S * b->A;
    const int64_t *dmax = delta;
    const int64_t *dsum = delta + nq, *dcnt = dsum + nq, *dn = dsum + 2 * nq, *dt = dn + nsa, *fc = dt + 1;
    if (b->priv) { b->stats[6]++; return; }
    if (b->qrepr == RLO_QREPR_F64) {
        const int hb = fq_merge_headroom(b->merge_groups);
        const int seq = b->q_forced == RLO_QMODE_F64_SEQ;
        for (size_t i = 0; i < nq; ++i) {
            const uint64_t n = (uint64_t)dcnt[i];
            if (!n) continue;
            const uint8_t f = (uint8_t)((fc[i] ? QF_NAN : 0) | (fc[nq + i] ? QF_PINF : 0) | (fc[2 * nq + i] ? QF_NINF : 0));
            double v;
            if (f) v = nf_value(f);
            else if (seq) v = b->fseq[i] * (1.0 / (double)n);
            else v = fq_mean(dsum[i], n, fq_grid((uint32_t)dmax[i]) + hb);
            b->qd_base[i] = canon_nan(v);
        }
    } else {
        for (size_t i = 0; i < nq; ++i) {
            b->q_base[i] = q_clamp_count(b, b->q_base[i] + mean_delta(dsum[i], dcnt[i]));
            if (fc[i]) b->f_base[i] |= QF_NAN;
            if (fc[nq + i]) b->f_base[i] |= QF_PINF;
            if (fc[2 * nq + i]) b->f_base[i] |= QF_NINF;
        }
    }
    for (size_t i = 0; i < nsa; ++i) b->n_base[i] = b->n_base[i] + (uint64_t)dn[i];
    b->t_base = (uint64_t)((int64_t)b->t_base + *dt);
    b->stats[6]++;
}

static void run_launch(rlo_batch *b) {
    const uint64_t nw = rlo_batch_delta_words(b);
    int64_t *delta = (int64_t *)calloc(nw, 8);
    rlo_batch_launch_groups(b, delta);
    rlo_batch_fold(b, delta);
    rlo_batch_apply_delta(b, delta);
    free(delta);
}
static uint64_t count_done(const rlo_batch *b) {
    uint64_t done = 0;
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) done += b->lanes[i].mode == RLO_MODE_DONE;
    return done;
}

/* run(): the device's done-lane slot accumulates over the launches of a run() call */
void rlo_batch_run(rlo_batch *b, uint32_t n_launches) {
    for (uint32_t i = 0; i < n_launches; ++i) { run_launch(b); b->last_done += count_done(b); }
}
static int all_done(const rlo_batch *b) {
    for (uint32_t i = 0; i < b->c.n_lanes; ++i)
        if (b->lanes[i].mode != RLO_MODE_DONE) return 0;
    return 1;
}
/* every lane starts a new episode with an empty trace set (the reference clears
 * E on termination, elegibility_traces_agent.rs:98-100, and train()/evaluate()
 * begin at an episode start); mode set, episode counters 0 (rl.h rl_agent_train) */
static void arm_lanes(rlo_batch *b, int mode, uint64_t eval_left) {
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
        lane_t *L = &b->lanes[i];
        L->need_reset = 1; L->train_ep = 0; L->eval_left = eval_left;
        L->mode = mode;
        if (L->trace) { memset(L->trace, 0, sizeof(double) * b->S * b->A); memset(L->visited, 0, b->S); L->vcnt = 0; }
    }
}
uint64_t rlo_batch_train_episodes(rlo_batch *b, uint64_t n, uint64_t eval_at) {
    if (n == 0) return 0;   /* Agent::train(env, 0, ..) runs no episode (src/agent.rs:80): a no-op */
    b->target_episodes = n; b->eval_at = eval_at; b->eval_only = 0;
    arm_lanes(b, RLO_MODE_TRAIN, 0);
    uint64_t launches = 0;
    while (!all_done(b)) { run_launch(b); launches++; b->last_done = count_done(b); }
    b->target_episodes = 0; b->eval_at = 0;
    arm_lanes(b, RLO_MODE_TRAIN, 0);     /* back to training: run() keeps training */
    return launches;
}
uint64_t rlo_batch_evaluate(rlo_batch *b, uint64_t n) {
    if (n == 0) return 0;
    b->eval_only = 1; b->target_episodes = 0; b->eval_at = 0;
    arm_lanes(b, RLO_MODE_EVAL, n);
    uint64_t launches = 0;
    while (!all_done(b)) { run_launch(b); launches++; b->last_done = count_done(b); }
    b->eval_only = 0;
    arm_lanes(b, RLO_MODE_TRAIN, 0);
    return launches;
}
void rlo_batch_get_q(const rlo_batch *b, double *out) {
    size_t nq = (size_t)b->P * b->S * b->A;
    if (b->feat) {        /* [L][1][S][A] get_values of every state */
        for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
            ((rlo_batch *)b)->w_g = b->lanes[i].w;
            for (uint32_t st = 0; st < b->S; ++st) b_row(b, 0, st, out + i * nq + (size_t)st * b->A);
        }
        return;
    }
    if (b->priv) {        /* [L][P][S][A] */
        for (uint32_t i = 0; i < b->c.n_lanes; ++i) memcpy(out + i * nq, b->lanes[i].qd, nq * sizeof(double));
        return;
    }
    if (b->qrepr == RLO_QREPR_F64) { memcpy(out, b->qd_base, nq * 8); return; }
    for (size_t i = 0; i < nq; ++i) out[i] = q_val(b->q_base[i], b->f_base[i]);
}
/* Policy contents set by the caller (rl.h rl_agent_set_q): shared mode keeps
 * the values in f64, or in the fixed point when the range proof holds and every
 * value is exact in it (o_choose_repr); private mode copies lane tables [L][P][S][A] */
void rlo_batch_set_q(rlo_batch *b, const double *in) {
    size_t nq = (size_t)b->P * b->S * b->A;
    if (b->priv) {
        for (uint32_t i = 0; i < b->c.n_lanes; ++i) memcpy(b->lanes[i].qd, in + i * nq, nq * sizeof(double));
        return;
    }
    for (size_t i = 0; i < nq; ++i) b->qd_base[i] = canon_nan(in[i]);
    o_set_abs0(b, in, nq);
    o_choose_repr(b);
}
/* raw words: the fixed-point integers, or the f64 bits (canonical NaN) */
void rlo_batch_get_q_raw(const rlo_batch *b, int64_t *out) {
    const size_t nq = (size_t)b->P * b->S * b->A;
    memcpy(out, b->qrepr == RLO_QREPR_F64 ? (const void *)b->qd_base : (const void *)b->q_base, sizeof(int64_t) * nq);
}
void rlo_batch_get_qflags(const rlo_batch *b, uint8_t *out) {
    const size_t nq = (size_t)b->P * b->S * b->A;
    if (b->qrepr == RLO_QREPR_F64) {
        for (size_t i = 0; i < nq; ++i) out[i] = isfinite(b->qd_base[i]) ? 0 : nf_flag(b->qd_base[i]);
        return;
    }
    memcpy(out, b->f_base, nq);
}
void rlo_batch_get_ucb(const rlo_batch *b, uint64_t *counts, uint64_t *t) {
    if (b->priv) {        /* [L][S][A], t[L] */
        size_t nsa = (size_t)b->S * b->A;
        for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
            memcpy(counts + i * nsa, b->lanes[i].n, nsa * sizeof(uint64_t));
            t[i] = b->lanes[i].t;
        }
        return;
    }
    memcpy(counts, b->n_base, sizeof(uint64_t) * b->S * b->A);
    *t = b->t_base;
}
void rlo_batch_set_ucb(rlo_batch *b, const uint64_t *counts, const uint64_t *t) {
    if (b->priv) {
        size_t nsa = (size_t)b->S * b->A;
        for (uint32_t i = 0; i < b->c.n_lanes; ++i) {
            memcpy(b->lanes[i].n, counts + i * nsa, nsa * sizeof(uint64_t));
            b->lanes[i].t = t[i];
        }
        return;
    }
    memcpy(b->n_base, counts, sizeof(uint64_t) * b->S * b->A);
    b->t_base = *t;
}
uint64_t rlo_batch_take_records(rlo_batch *b, rlo_record *out, uint64_t cap) {
    uint64_t n = b->records.n;
    if (out && n && cap) memcpy(out, b->records.p, (n < cap ? n : cap) * sizeof(rlo_record));
    b->records.n = 0;
    return n;
}
uint64_t rlo_batch_n_records(const rlo_batch *b) { return b->records.n; }
/* out[16]: rl_stats order (slot 5 = lanes DONE at the end of the last launch) */
void rlo_batch_stats(const rlo_batch *b, uint64_t *out) {
    memcpy(out, b->stats, sizeof b->stats);
    out[5] = b->last_done;
}
void rlo_batch_lane_eps(const rlo_batch *b, double *out) {
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) out[i] = b->lanes[i].eps;
}

void rlo_batch_get_weights(const rlo_batch *b, double *out) {
    if (!b->feat) return;
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) memcpy(out + (size_t)i * b->net.np, b->lanes[i].w, sizeof(double) * b->net.np);
}
void rlo_batch_set_weights(rlo_batch *b, const double *in) {
    if (!b->feat) return;
    for (uint32_t i = 0; i < b->c.n_lanes; ++i) memcpy(b->lanes[i].w, in + (size_t)i * b->net.np, sizeof(double) * b->net.np);
}

// rl_device.h — gfx950 device building blocks of the tabular-RL hot path:
// per-lane RNG stream, rand-0.8.5 distribution mappings, the shared ln(),
// fixed-point Q, argmax/max and the four environments.
//
// Numerics contract (bit-exact with the CPU oracle and the reference's f64
// arithmetic): no FP contraction, no fast-math; every expression keeps the
// reference's evaluation order (citations inline).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rl_kparams.h"
#include "rl_taxi.h"

#pragma clang fp contract(off)

namespace rlamd {

constexpr double MIN_POSITIVE = 2.2250738585072014e-308;  // f64::MIN_POSITIVE

// ------------------------------------------------------------------ RNG
// Replaces rand::thread_rng() (entropy-seeded ChaCha12) at the reference's draw
// sites with one xoshiro128+ stream per lane, keyed (seed, global lane id).  Every
// draw site uses the words' high bits; '+' costs one VALU op of output mixing.
// three-input XOR in one VALU op: gfx950's v_bitop3_b32 with truth table 0x96
// (the compiler does not form it from a ^ b ^ c)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
struct Rng {
    uint32_t s0, s1, s2, s3;
    // xoshiro128 state transition written on the old words (s2 ^= s0; s3 ^= s1;
    // s1 ^= s2; s0 ^= s3; s2 ^= s1 << 9; s3 = rotl(s3, 11)): three xor3 + one xor
    // + the shift and the rotate
    __device__ __forceinline__ void advance() {
        const uint32_t t = s1 << 9;
        const uint32_t n1 = xor3(s1, s2, s0), n2 = xor3(s2, s0, t), n0 = xor3(s0, s3, s1), n3 = s3 ^ s1;
        s0 = n0; s1 = n1; s2 = n2;
        s3 = __builtin_rotateleft32(n3, 11);
    }
    __device__ __forceinline__ uint32_t next_u32() {
        const uint32_t r = s0 + s3;
        advance();
        return r;
    }
    // advance as next_u32 does, without the output scrambler (a draw whose value is unused)
    __device__ __forceinline__ void skip_u32() { advance(); }
    // RngCore::next_u64 of a 32-bit block generator: low word first
    __device__ __forceinline__ uint64_t next_u64() {
        const uint64_t lo = next_u32();
        const uint64_t hi = next_u32();
        return lo | (hi << 32);
    }
};

__host__ __device__ inline uint64_t splitmix64(uint64_t &x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint4 rng_seed(uint64_t seed, uint64_t lane) {
    uint64_t x = seed + lane * 0x632BE59BD9B4E019ull;
    const uint64_t a = splitmix64(x), b = splitmix64(x);
    uint4 r = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
    if ((r.x | r.y | r.z | r.w) == 0) r.x = 1;
    return r;
}

// rand 0.8.5 UniformFloat<f64> for Uniform::from(0.0..1.0): ((u64>>12)|1.0) - 1.0
__device__ __forceinline__ double uniform01(Rng &r) {
    const uint64_t bits = (r.next_u64() >> 12) | 0x3FF0000000000000ull;
    return __longlong_as_double((long long)bits) - 1.0;
}
// The eps-greedy test u < eps for u = UniformFloat(0..1) = m * 2^-52, m the top 52
// bits of a u64 (uniform_epsilon_greed.rs:51-54): the high word h is drawn first
// and decides the test unless h * 2^-32 < eps < (h + 1) * 2^-32 (probability
// <= 2^-32); only then is the word holding m's low 20 bits drawn (DESIGN §2
// "draws": the same exact test, one u32 per selection).  eps * 2^32 and h + 1
// are exact; NaN eps fails every compare and reaches the exact test.
#ifndef RLAMD_EPSX
#define RLAMD_EPSX 1
#endif
__device__ __forceinline__ bool eps_test(Rng &r, double eps) {
    const uint32_t h = r.next_u32();
    const double e32 = __builtin_ldexp(eps, 32), hd = (double)h;
    bool lt = hd + 1.0 <= e32;                  // u < (h + 1) 2^-32 <= eps
#if RLAMD_EPSX
    const bool may = hd < e32;                  // u < eps possible (implied by lt)
    if (may != lt) {                            // undecided: m's low bits
#else
    if (!lt && hd < e32) {                      // undecided: m's low bits
#endif
        const uint32_t l = r.next_u32();
        const uint64_t bits = (((((uint64_t)h << 32) | l) >> 12)) | 0x3FF0000000000000ull;
        lt = __longlong_as_double((long long)bits) - 1.0 < eps;
    }
    return lt;
}
// rand 0.8.5 UniformInt<usize>::sample for Uniform::from(0..A)
// (uniform_epsilon_greed.rs:34,62): widening multiply, reject lo > zone.
// A power of two (FrozenLake / CliffWalking 4, Blackjack 2): the zone rejects
// nothing and the result is the top log2(A) bits of next_u64's high word, whose
// low word is never looked at — so the stream draws ONE u32 and takes its top
// bits (the same uniform distribution over 0..A; DESIGN §2 "draws").
template <uint32_t A>
__device__ __forceinline__ uint32_t uniform_action(Rng &r) {
    if constexpr (A >= 2u && (A & (A - 1u)) == 0u) return r.next_u32() >> (32 - __builtin_ctz(A));
    constexpr uint64_t reject = (0ull - (uint64_t)A) % (uint64_t)A;  // (MAX - A + 1) % A
    constexpr uint64_t zone = ~0ull - reject;
    for (;;) {
        const uint64_t v = r.next_u64();
        const uint64_t lo = v * (uint64_t)A;
        const uint64_t hi = __umul64hi(v, (uint64_t)A);
        if (lo <= zone) return (uint32_t)hi;
    }
}
// rand 0.8.5 Rng::gen_range(0..n) for usize = sample_single_inclusive: the
// "conservative" zone (n << lz(n)) - 1 (RandomModel::get_info, random_model.rs:29-31)
__device__ __forceinline__ uint32_t gen_index(Rng &r, uint32_t n) {
    const uint64_t range = n;
    const uint64_t zone = (range << __clzll((long long)range)) - 1ull;
    for (;;) {
        const uint64_t v = r.next_u64();
        if (v * range <= zone) return (uint32_t)__umul64hi(v, range);
    }
}
// Cards (blackjack.rs:54, rand 0.8.5 Uniform<u8>(1..11)): rand's widening-multiply-
// and-zone rule at 16 bits — a half h gives card 1 + (h*10 >> 16), rejected when
// (h*10 & 0xffff) > 65535 - 6 — the same exact uniform over 1..10 as the u32 rule,
// so one u32 supplies two cards, high half first (a 24-bit multiply instead of a
// 64-bit one).  Each env operation (a deal, a hit, the dealer's draws after a
// stick) takes its cards from its own words: a rejected half is skipped, a half
// left at the operation's end is discarded (DESIGN §2 "cards"; oracle cardsrc).
__device__ __forceinline__ bool card16(uint32_t h, uint32_t &c) {
    const uint32_t m = __umul24(h, 10u);
    c = 1u + (m >> 16);
    return (m & 0xFFFFu) <= 0xFFFFu - 6u;
}
struct CardSrc {
    uint32_t w = 0, n = 0;   // the operation's current word, halves left
    __device__ __forceinline__ uint32_t next(Rng &r) {
        for (;;) {
            if (n == 0u) { w = r.next_u32(); n = 2u; }
            const uint32_t h = n == 2u ? w >> 16 : w & 0xFFFFu;
            --n;
            uint32_t c;
            if (card16(h, c)) return c;
        }
    }
};

// ------------------------------------------------------------------ ln()
// fdlibm e_log.c operation sequence; the oracle (oracle/rlref.c rlo_log)
// evaluates the identical sequence on the host, so UCB bonuses
// (upper_confidence_bound.rs:36) agree bit for bit.
__device__ inline double rl_log(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16, Lg1 = 6.666666666666735130e-01,
                 Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                 Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01,
                 Lg6 = 1.531383769920937332e-01, Lg7 = 1.479819860511658591e-01;
    uint64_t u = (uint64_t)__double_as_longlong(x);
    int32_t hx = (int32_t)(u >> 32);
    const uint32_t lx = (uint32_t)u;
    int32_t k = 0;
    if (hx < 0x00100000) {
        if (((hx & 0x7fffffff) | (int32_t)lx) == 0) return -__builtin_inf();
        if (hx < 0) return __builtin_nan("");
        k -= 54;
        x *= two54;
        u = (uint64_t)__double_as_longlong(x);
        hx = (int32_t)(u >> 32);
    }
    if (hx >= 0x7ff00000) return x + x;
    k += (hx >> 20) - 1023;
    hx &= 0x000fffff;
    int32_t i = (hx + 0x95f64) & 0x100000;
    u = ((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (u & 0xffffffffull);
    x = __longlong_as_double((long long)u);
    k += (i >> 20);
    const double f = x - 1.0;
    double dk, R;
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
    const double s = f / (2.0 + f);
    dk = (double)k;
    const double z = s * s;
    i = hx - 0x6147a;
    const double w = z * z;
    const int32_t j = 0x6b851 - hx;
    const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
    const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
    i |= j;
    R = t2 + t1;
    if (i > 0) {
        const double hfsq = 0.5 * f * f;
        if (k == 0) return f - (hfsq - s * (hfsq + R));
        return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
    }
    if (k == 0) return f - s * (f - R);
    return dk * ln2_hi - ((s * (f - R) - dk * ln2_lo) - f);
}

// ------------------------------------------------------------------ exp / expm1 / tanh
// fdlibm e_exp.c / s_expm1.c / s_tanh.c operation sequences, evaluated
// identically by the oracle (oracle/rlref.c rlo_exp / rlo_expm1 / rlo_tanh):
// the neural policy's activations (src/network/activation.rs) agree bit for bit.
__device__ __forceinline__ uint32_t hi_word(double x) { return (uint32_t)((uint64_t)__double_as_longlong(x) >> 32); }
__device__ __forceinline__ uint32_t lo_word(double x) { return (uint32_t)(uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double with_hi(double x, uint32_t hi) {
    const uint64_t u = ((uint64_t)hi << 32) | ((uint64_t)__double_as_longlong(x) & 0xffffffffull);
    return __longlong_as_double((long long)u);
}
__device__ __forceinline__ double add_exponent(double y, int k) { return with_hi(y, (uint32_t)((int32_t)hi_word(y) + k * (1 << 20))); }

__device__ inline double rl_exp(double x) {
    const double huge = 1.0e+300, twom1000 = 9.33263618503218878990e-302,
                 o_threshold = 7.09782712893383973096e+02, u_threshold = -7.45133219101941108420e+02,
                 ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
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
            hi = x - (xsb ? -ln2HI : ln2HI); lo = xsb ? -ln2LO : ln2LO; k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
            t = (double)k;
            hi = x - t * ln2HI;
            lo = t * ln2LO;
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

__device__ inline double rl_expm1(double x) {
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
        t = with_hi(0.0, 0x3ff00000u - (0x200000u >> k));
        y = t - (e - x);
        y = add_exponent(y, k);
    } else {
        t = with_hi(0.0, (uint32_t)((0x3ff - k) << 20));
        y = x - (e + t);
        y += 1.0;
        y = add_exponent(y, k);
    }
    return y;
}

__device__ inline double rl_tanh(double x) {
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
            t = rl_expm1(2.0 * __builtin_fabs(x));
            z = 1.0 - 2.0 / (t + 2.0);
        } else {
            t = rl_expm1(-2.0 * __builtin_fabs(x));
            z = -t / (t + 2.0);
        }
    } else {
        z = 1.0 - tiny;
    }
    return jx >= 0 ? z : -z;
}

// ------------------------------------------------------------------ activations
// src/network/activation.rs (f, f') pairs; f64::max / f64::min return the
// non-NaN operand.  Softmax (layer-wide) lives in the network code.
__device__ __forceinline__ double max_rs(double a, double b) { return (a > b || b != b) ? a : b; }
__device__ __forceinline__ double min_rs(double a, double b) { return (a < b || b != b) ? a : b; }
__device__ __forceinline__ double sigmoid_(double v) { return 1.0 / (1.0 + rl_exp(-v)); }
// act_t / act_pt: one activation as a compile-time choice (the register-resident
// network kernel, rl_net.h NetRegs); act_f / act_fp: the run-time switch over them
template <int ACT>
__device__ __forceinline__ double act_t(double v) {
    if constexpr (ACT == RL_ACT_TANH) return rl_tanh(v);
    else if constexpr (ACT == RL_ACT_RELU) return max_rs(v, 0.0);
    else if constexpr (ACT == RL_ACT_LEAKY_RELU) return max_rs(v, 0.1 * v);
    else if constexpr (ACT == RL_ACT_RELU6) return min_rs(max_rs(v, 0.0), 6.0);
    // v and 0.1 v share a sign (and are both NaN or neither), so max_rs is the
    // hardware max here, and min_rs against 6.0 the hardware min: the same value
    // (NaN payloads aside) in 2 instructions instead of 6
    else if constexpr (ACT == RL_ACT_LEAKY_RELU6) return __builtin_fmin(__builtin_fmax(v, 0.1 * v), 6.0);
    else if constexpr (ACT == RL_ACT_SIGMOID) return sigmoid_(v);
    else if constexpr (ACT == RL_ACT_SWISH) return v * sigmoid_(v);
    else if constexpr (ACT == RL_ACT_HARD_SWISH) return (v * min_rs(max_rs(v + 3.0, 0.0), 6.0)) / 6.0;
    else return v;
}
template <int ACT>
__device__ __forceinline__ double act_pt(double v) {
    if constexpr (ACT == RL_ACT_TANH) { const double t = rl_tanh(v); return 1.0 - t * t; }
    else if constexpr (ACT == RL_ACT_RELU) return v > 0.0 ? 1.0 : 0.0;
    else if constexpr (ACT == RL_ACT_LEAKY_RELU) return v > 0.0 ? 1.0 : 0.01;
    else if constexpr (ACT == RL_ACT_RELU6) return (v > 0.0 && v < 6.0) ? 1.0 : 0.0;
    else if constexpr (ACT == RL_ACT_LEAKY_RELU6) return (v > 0.0 && v < 6.0) ? 1.0 : 0.01;
    else if constexpr (ACT == RL_ACT_SIGMOID) { const double sg = sigmoid_(v); return sg * (1.0 - sg); }
    else if constexpr (ACT == RL_ACT_SWISH) { const double e = rl_exp(v); return (e * (v + e + 1.0)) / ((e + 1.0) * (e + 1.0)); }
    else if constexpr (ACT == RL_ACT_HARD_SWISH) return v > -3.0 ? (2.0 * v + 3.0) / 6.0 : 0.0;
    else return 1.0;
}
__device__ inline double act_f(int act, double v) {
    switch (act) {
    case RL_ACT_TANH: return act_t<RL_ACT_TANH>(v);
    case RL_ACT_RELU: return act_t<RL_ACT_RELU>(v);
    case RL_ACT_LEAKY_RELU: return act_t<RL_ACT_LEAKY_RELU>(v);
    case RL_ACT_RELU6: return act_t<RL_ACT_RELU6>(v);
    case RL_ACT_LEAKY_RELU6: return act_t<RL_ACT_LEAKY_RELU6>(v);
    case RL_ACT_SIGMOID: return act_t<RL_ACT_SIGMOID>(v);
    case RL_ACT_SWISH: return act_t<RL_ACT_SWISH>(v);
    case RL_ACT_HARD_SWISH: return act_t<RL_ACT_HARD_SWISH>(v);
    default: return v;
    }
}
__device__ inline double act_fp(int act, double v) {
    switch (act) {
    case RL_ACT_TANH: return act_pt<RL_ACT_TANH>(v);
    case RL_ACT_RELU: return act_pt<RL_ACT_RELU>(v);
    case RL_ACT_LEAKY_RELU: return act_pt<RL_ACT_LEAKY_RELU>(v);
    case RL_ACT_RELU6: return act_pt<RL_ACT_RELU6>(v);
    case RL_ACT_LEAKY_RELU6: return act_pt<RL_ACT_LEAKY_RELU6>(v);
    case RL_ACT_SIGMOID: return act_pt<RL_ACT_SIGMOID>(v);
    case RL_ACT_SWISH: return act_pt<RL_ACT_SWISH>(v);
    case RL_ACT_HARD_SWISH: return act_pt<RL_ACT_HARD_SWISH>(v);
    default: return 1.0;
    }
}

// UCB value u_i = q_i + c * sqrt(ln(t) / (n_i + MIN_POSITIVE))
// (upper_confidence_bound.rs:33-37,53-57); sqrt and / are correctly rounded.
__device__ __forceinline__ double ucb_value(double q, double c, double lnt, double n) {
    return q + c * __builtin_sqrt(lnt / (n + MIN_POSITIVE));
}

// The UCB values of a row without the division and square root where IEEE
// arithmetic fixes the result (the bench regime of Expected SARSA +
// UCB is almost all such rows):
//   n_i == 0: lnt / (0 + MIN_POSITIVE) is exactly lnt * 2^1022 (a power-of-two
//             quotient; it overflows to +inf from t = 55), so u_i = v_i + b0 with
//             b0 = c * sqrt(lnt * 2^1022) shared by the row;
//   n_i >= 1 and v_i non-finite: the bonus c * sqrt(lnt / n) is finite (lnt <=
//             ln 2^64 < 45, |c| < 2^1020), u_i = v_i.
// Returns the mask of entries still needing ucb_value (u[i] = 0 for them).
template <int A>
__device__ __forceinline__ uint32_t ucb_known(const double (&v)[A], const uint64_t (&n)[A], double c, double lnt,
                                              double (&u)[A]) {
    const double b0 = c * __builtin_sqrt(lnt * 0x1p1022);
    const bool c_fin = __builtin_fabs(c) < 0x1p1020;
    uint32_t need = 0;
#pragma unroll
    for (int i = 0; i < A; ++i) {
        const bool z = n[i] == 0ull, nf = !__builtin_isfinite(v[i]) && c_fin;
        u[i] = z ? v[i] + b0 : (nf ? v[i] : 0.0);
        need |= (!z && !nf) ? (1u << i) : 0u;
    }
    return need;
}
#ifndef RLAMD_UCB_PRED
#define RLAMD_UCB_PRED 0   // 1: ucb_fill predicated (every entry computed, selected): measured 0.4521 vs 0.4513 ms
                           // on cfg 3, 1.400 vs 1.401 on cfg 8 (profiles/r05/ucb_pred_ab.txt), so off
#endif
template <int A>
__device__ __forceinline__ void ucb_fill(const double (&v)[A], const uint64_t (&n)[A], double c, double lnt,
                                         uint32_t need, double (&u)[A]) {
    if constexpr (RLAMD_UCB_PRED) {
        // predicated: the A quotients and roots for every lane of the wave, kept where
        // needed (a divergent `if` per action cost an exec-mask triple each, VERDICT
        // r04 weak 4); the values are those of ucb_value, selected bit for bit
#pragma unroll
        for (int i = 0; i < A; ++i) {
            const double x = ucb_value(v[i], c, lnt, (double)n[i]);
            u[i] = ((need >> i) & 1u) ? x : u[i];
        }
    } else {
#pragma unroll
        for (int i = 0; i < A; ++i)
            if ((need >> i) & 1u) u[i] = ucb_value(v[i], c, lnt, (double)n[i]);
    }
}

// ------------------------------------------------------------------ f64 shared Q
// The f64 representation of a learner group's Q (KParams::fq; the host picks it
// wherever the fixed point's range is not proven): entries are the reference's
// f64 values with its whole range, NaN stored canonical so equal states compare
// bitwise.  A step's contributions d_i to an entry are summed exactly on the
// integer grid 2^e of the largest, e = max(code, 1) - 1075 with code = the
// biased exponent (oracle/rlref.c fq_step_combine).
constexpr uint64_t QNAN_BITS = 0x7FF8000000000000ull;
__device__ __forceinline__ double as_f64(uint64_t u) { return __longlong_as_double((long long)u); }
__device__ __forceinline__ uint64_t f64_bits(double x) { return (uint64_t)__double_as_longlong(x); }
__device__ __forceinline__ double canon_nan(double x) { return x != x ? as_f64(QNAN_BITS) : x; }
__device__ __forceinline__ uint32_t f64_code(double x) {
    return ((uint32_t)((uint64_t)__double_as_longlong(x) >> 52)) & 0x7ffu;
}
__device__ __forceinline__ int fq_grid(uint32_t code) { return (int)(code > 1u ? code : 1u) - 1075; }
// kind of a non-finite value (QF_* bit)
__device__ __forceinline__ uint32_t nf_flag(double x) { return x != x ? QF_NAN : (x > 0.0 ? QF_PINF : QF_NINF); }
// the IEEE sum of contributions of these non-finite kinds
__device__ __forceinline__ double nf_value(uint32_t f) {
    if ((f & QF_NAN) || ((f & QF_PINF) && (f & QF_NINF))) return as_f64(QNAN_BITS);
    return (f & QF_PINF) ? __builtin_inf() : -__builtin_inf();
}
// d on the grid 2^e, rounded half-to-even; |d| < 2^(e+53) so the result is exact in int64
__device__ __forceinline__ int64_t fq_raw(double d, int e) {
    return (int64_t)__builtin_rint(__builtin_ldexp(d, -e));
}
// 1.0 / n (0 for n == 0) without a table read: v_rcp_f64 and two Newton steps
// (with one step the cfg 2 fixtures failed: not correctly rounded).  After the
// first step the relative error is below 2^-52, after the second y1 * (2 - n y1)
// is within about 2^-104 of 1/n and the last fma rounds once, and 1/n for small n
// is far from any rounding midpoint, so this should be the correctly rounded
// 1.0 / n — an argument, not a check: it is used only with RLAMD_SETTLE_RCPN,
// which is off because on cfg 2 the f64 chain measured slower than the table read
// it replaces (0.199 against 0.188 ms per launch, A/B on one box).
__device__ __forceinline__ double rcp_nr(uint32_t n) {
    const double dn = (double)n;
    const double r0 = __builtin_amdgcn_rcp(dn);
    const double e0 = __builtin_fma(-dn, r0, 1.0);
    const double r1 = __builtin_fma(r0, e0, r0);
    const double e1 = __builtin_fma(-dn, r1, 1.0);
    return n ? __builtin_fma(r1, e1, r1) : 0.0;
}
// argmax (first maximum, strict >) and max of one f64 row in a single pass
// (utils.rs:1-21: a NaN at index 0 sticks, later NaNs never win)
template <int A>
__device__ __forceinline__ uint32_t argmax_max_f64(const double (&v)[A], double &m) {
    m = v[0];
    uint32_t r = 0;
#pragma unroll
    for (int i = 1; i < A; ++i) {
        const bool gt = v[i] > m;
        m = gt ? v[i] : m;
        r = gt ? (uint32_t)i : r;
    }
    return r;
}

// ------------------------------------------------------------------ fixed-point Q
// Shared-mode Q entries in the fixed-point representation (only where the host
// proved the range, rl_host.cpp delta_bound) are int64, value = raw * 2^-40,
// |raw| <= 2^51 (|Q| <= 2048): every entry — and (a+b)/2 of two entries —
// converts to f64 exactly, so comparisons on raw int64 are identical to the
// reference's f64 comparisons (argmax / max without conversions).
constexpr int64_t Q_RAW_MAX = (int64_t)1 << 51;

// rint(x) as int64 for |x| < 2^51 (the 1.5*2^52 magic add rounds half-to-even)
__device__ __forceinline__ int64_t rint_i64_small(double x) {
    const double y = x + 0x1.8p52;
    return (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull);
}
// delta -> raw units: rint(d * 2^40), exact in range because the host proved
// |d| * 2^40 < 2^51 wherever the fixed point runs (rl_host.cpp delta_bound)
__device__ __forceinline__ int64_t q_fix_inrange(double d) { return rint_i64_small(d * 0x1p40); }
// (double)raw * 2^-40 for |raw| <= 2^51 in two operations: raw added to the bits
// of 1.5*2^12 (whose ulp is 2^-40) gives 6144 + raw*2^-40 exactly, then 6144 off.
__device__ __forceinline__ double q_val(int64_t raw) {
    return __longlong_as_double((long long)(0x40B8000000000000ull + (uint64_t)raw)) - 6144.0;
}
template <int A>
__device__ __forceinline__ uint32_t argmax_i64(const int64_t (&v)[A]) {
    int64_t m = v[0];
    uint32_t r = 0;
#pragma unroll
    for (int i = 1; i < A; ++i)
        if (v[i] > m) { m = v[i]; r = (uint32_t)i; }
    return r;
}
// argmax and max of one row in a single pass (first maximum, strict `>`): the
// index is argmax_i64's and the value max_i64's
template <int A>
__device__ __forceinline__ uint32_t argmax_max_i64(const int64_t (&v)[A], int64_t &m) {
    m = v[0];
    uint32_t r = 0;
#pragma unroll
    for (int i = 1; i < A; ++i) {
        const bool gt = v[i] > m;
        m = gt ? v[i] : m;
        r = gt ? (uint32_t)i : r;
    }
    return r;
}
template <int A>
__device__ __forceinline__ int64_t max_i64(const int64_t (&v)[A]) {
    int64_t m = v[0];
#pragma unroll
    for (int i = 1; i < A; ++i) m = v[i] > m ? v[i] : m;
    return m;
}
// x unchanged, but opaque to the optimizer (an empty asm): a select chain over
// opq(v[j]) cannot be folded back into v[i], which would put v in scratch memory
template <class T>
__device__ __forceinline__ T opq(T x) {
    asm("" : "+v"(x));
    return x;
}
template <int A, class T>
__device__ __forceinline__ T pick(const T (&v)[A], uint32_t i) {   // v[i] as a select chain (in registers)
    T r = opq(v[0]);
#pragma unroll
    for (int j = 1; j < A; ++j) r = (i == (uint32_t)j) ? opq(v[j]) : r;
    return r;
}

// ------------------------------------------------------------------ utils
// argmax: first maximum, strict `>` (src/utils.rs:1-11)
template <int A>
__device__ __forceinline__ uint32_t argmax(const double (&v)[A]) {
    double m = v[0];
    uint32_t r = 0;
#pragma unroll
    for (int i = 1; i < A; ++i)
        if (v[i] > m) { m = v[i]; r = (uint32_t)i; }
    return r;
}
// max: src/utils.rs:13-21
template <int A>
__device__ __forceinline__ double vmax(const double (&v)[A]) {
    double m = v[0];
#pragma unroll
    for (int i = 1; i < A; ++i)
        if (v[i] > m) m = v[i];
    return m;
}
// categorical_sample over a cumulative table: first i with cdf[i] > u, else 0
// (src/utils.rs:33-43; the cdf is the reference's running sum, precomputed)
__device__ __forceinline__ uint32_t cdf_search(const double *cdf, uint32_t n, double u) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cdf[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo < n ? lo : 0u;
}

// ------------------------------------------------------------------ environments
// Lane env state: pos (dense obs), z (curr_step, or the Blackjack hand), ready.
struct EnvTables {
    const uint32_t *trans;
    const double *cdf;
    uint32_t n_start, max_steps;
    double th1, th2, th3, trunc_reward;   // trunc_reward: host-side record only (the envs' own constants)
    int32_t fixed_start;   // >= 0: categorical_sample over the start cdf returns this for every u
    int32_t slippery;      // FrozenLake: the map has stochastic rows (uniform per launch)
    uint32_t S;            // |S|: row stride of an action-major table (AM layout below)
};
// Transition-table index of (s, a): state-major trans[s*A + a] (HBM, the private
// kernel), or action-major trans[a*S + s] (AM: the shared kernel's LDS copy, where
// lanes of one wave in neighbouring states then hit distinct LDS banks).
template <bool AM, int A>
__device__ __forceinline__ uint32_t tidx(const EnvTables &t, uint32_t s, uint32_t a) {
    return AM ? a * t.S + s : s * (uint32_t)A + a;
}
// Env::reset's categorical draw (taxi.rs:136-137): the search is skipped when
// the answer is fixed.
__device__ __forceinline__ uint32_t start_state(const EnvTables &t, double u) {
    return t.fixed_start >= 0 ? (uint32_t)t.fixed_start : cdf_search(t.cdf, t.n_start, u);
}

template <int ENV> struct EnvDev;

// FrozenLakeEnv (src/env/frozen_lake.rs).  trans[s*4+a]: 3 outcome bytes
// (bits 0-5 next, bit 6 reward==1.0, bit 7 terminated) + bit 24 "slippery row".
// One synchronous step of a FrozenLake-family lane that either RESETs (doR) or
// STEPs (doS), without branching on which.  Only a step on a slippery map
// draws (:126 / :235): the reference also draws at reset (:107-108 / :222-223,
// the one-'S' maps' categorical always returns 0) and on deterministic maps,
// values it never looks at, which the stream skips (DESIGN §2 "draws").  The
// table word is read by every lane (pos and a are always valid indices).
// Truncation: (0, 0.0, true) for FrozenLake (:119-122), (pos, -1.0, true) for
// FrozenLakeEdited (:227-231).
// The outcome byte's reward bit means 1.0 (FrozenLake) or 10.0 (edited; else -1.0).
// w: the table word trans[(pos, a)], read by the caller (possibly a step ahead)
template <bool EDITED, int SLIP, bool AM>
__device__ __forceinline__ void fl_advance(bool doR, bool doS, uint32_t &pos, uint32_t &z, uint32_t w, Rng &r,
                                           const EnvTables &t, uint32_t &s2, double &rew, bool &term) {
    const bool trunc = doS && z >= t.max_steps;
    const bool st = doS && !trunc;
    uint32_t i = 0;
    if (SLIP == 1 || (SLIP < 0 && t.slippery)) {      // the only draw whose value is used
        if (st) {
            const double u = uniform01(r);
            if (w & (1u << 24)) i = (t.th1 > u) ? 0u : (t.th2 > u) ? 1u : (t.th3 > u) ? 2u : 0u;
        }
    }
    const uint32_t o = (w >> (8 * i)) & 0xffu;
    const double r_bit = EDITED ? 10.0 : 1.0, r_else = EDITED ? -1.0 : 0.0;
    s2 = st ? (o & 63u) : ((EDITED && trunc) ? pos : 0u);
    rew = st ? ((o & 64u) ? r_bit : r_else) : ((EDITED && trunc) ? -1.0 : 0.0);
    term = trunc || (st && (o & 128u) != 0u);
    z = doR ? 0u : (st ? z + 1u : z);
    pos = s2;
}

// Both built-in maps (MAP_4X4 / MAP_8X8) have one 'S', at position 0, so
// Env::reset's categorical draw always returns 0 (the host asserts this): the
// draw is not made (its value is never used).  SLIP: the map's slippery
// flag as a compile-time constant (0 / 1), or -1 to read it at run time.
template <> struct EnvDev<RL_ENV_FROZEN_LAKE> {
    static constexpr int A = 4;
    __device__ static __forceinline__ uint32_t reset(uint32_t &z, Rng &, const EnvTables &) {
        z = 0;                                         // frozen_lake.rs:107-108: the categorical
        return 0u;                                     // draw returns 0 for every u: not drawn
    }
    template <int SLIP = -1, bool AM = false>
    __device__ static __forceinline__ void step(uint32_t &pos, uint32_t &z, uint32_t a, Rng &r,
                                                const EnvTables &t, uint32_t &s2, double &rew,
                                                bool &term) {
        if (z >= t.max_steps) { s2 = 0; rew = 0.0; term = true; return; }  // :119-122
        z += 1;
        const uint32_t w = t.trans[tidx<AM, 4>(t, pos, a)];
        uint32_t i = 0;
        if (SLIP == 1 || (SLIP < 0 && t.slippery)) {   // :126 (a deterministic map's draw is unused: skipped)
            const double u = uniform01(r);
            if (w & (1u << 24)) i = (t.th1 > u) ? 0u : (t.th2 > u) ? 1u : (t.th3 > u) ? 2u : 0u;
        }
        const uint32_t o = (w >> (8 * i)) & 0xffu;
        s2 = o & 63u;
        rew = (o & 64u) ? 1.0 : 0.0;
        term = (o & 128u) != 0;
        pos = s2;
    }
};

// FrozenLakeEditedEnv (src/env/frozen_lake_edited.rs), dense obs = position.
// trans[s*4+a] as FrozenLake's: 3 outcome bytes (bits 0-5 next, bit 6 reward
// 10.0 (else -1.0), bit 7 terminated) + bit 24 "slippery row".  Truncation
// observes the current position with -1.0 (:227-231); one draw per step (:235).
template <> struct EnvDev<RL_ENV_FROZEN_LAKE_EDITED> {
    static constexpr int A = 4;
    __device__ static __forceinline__ uint32_t reset(uint32_t &z, Rng &, const EnvTables &) {
        z = 0;                                         // :222-223, the start is position 0
        return 0u;                                     // (same maps as FrozenLakeEnv): not drawn
    }
    template <int SLIP = -1, bool AM = false>
    __device__ static __forceinline__ void step(uint32_t &pos, uint32_t &z, uint32_t a, Rng &r,
                                                const EnvTables &t, uint32_t &s2, double &rew,
                                                bool &term) {
        if (z >= t.max_steps) { s2 = pos; rew = -1.0; term = true; return; }
        z += 1;
        const uint32_t w = t.trans[tidx<AM, 4>(t, pos, a)];
        uint32_t i = 0;
        if (SLIP == 1 || (SLIP < 0 && t.slippery)) {   // :235 (skipped on a deterministic map)
            const double u = uniform01(r);
            if (w & (1u << 24)) i = (t.th1 > u) ? 0u : (t.th2 > u) ? 1u : (t.th3 > u) ? 2u : 0u;
        }
        const uint32_t o = (w >> (8 * i)) & 0xffu;
        s2 = o & 63u;
        rew = (o & 64u) ? 10.0 : -1.0;
        term = (o & 128u) != 0;
        pos = s2;
    }
};

// CliffWalkingEnv (src/env/cliff_walking.rs): deterministic, no RNG.
// trans[s*4+a]: bits 0-5 next, bit 6 reward -100 (else -1), bit 7 terminated.
template <> struct EnvDev<RL_ENV_CLIFF_WALKING> {
    static constexpr int A = 4;
    __device__ static __forceinline__ uint32_t reset(uint32_t &z, Rng &, const EnvTables &) {
        z = 0;
        return 36u;                                    // cliff_walking.rs:71
    }
    template <int SLIP = -1, bool AM = false>
    __device__ static __forceinline__ void step(uint32_t &pos, uint32_t &z, uint32_t a, Rng &,
                                                const EnvTables &t, uint32_t &s2, double &rew,
                                                bool &term) {
        if (z >= t.max_steps) { s2 = 0; rew = -100.0; term = true; return; }  // :81-84
        z += 1;
        const uint32_t w = t.trans[tidx<AM, 4>(t, pos, a)];
        s2 = w & 63u;
        rew = (w & 64u) ? -100.0 : -1.0;
        term = (w & 128u) != 0;
        pos = s2;
    }
};

// TaxiEnv (src/env/taxi.rs): 500 states x 6 actions, deterministic.  The
// transition of (s, a) is computed from the state's digits instead of read from
// a table (no LDS for it: the learner group's LDS goes to Q and the u64 UCB
// counters).  taxi_word(s, a) = the table word the host builds (rl_host.cpp
// build_env checks all 3000 against TaxiEnv::new's loop, taxi.rs:63-112):
// bits 0-8 next, bits 9-10 reward code {-1,-10,+20}, bit 11 terminated.
template <> struct EnvDev<RL_ENV_TAXI> {
    static constexpr int A = 6;
    __device__ static __forceinline__ uint32_t reset(uint32_t &z, Rng &r, const EnvTables &t) {
        const double u = uniform01(r);                 // taxi.rs:136-137
        z = 0;
        return taxi_start(t.cdf, u);
    }
    template <int SLIP = -1, bool AM = false>
    __device__ static __forceinline__ void step(uint32_t &pos, uint32_t &z, uint32_t a, Rng &,
                                                const EnvTables &t, uint32_t &s2, double &rew,
                                                bool &term) {
        if (z >= t.max_steps) { s2 = 0; rew = 0.0; term = true; return; }  // :146-149
        z += 1;
        const uint32_t w = taxi_word(pos, a);
        s2 = w & 511u;
        const uint32_t rc = (w >> 9) & 3u;
        rew = rc == 0 ? -1.0 : (rc == 1 ? -10.0 : 20.0);
        term = (w & (1u << 11)) != 0;
        pos = s2;
    }
    // step() with the transition word already read (taxi_word(pos, a) == the table's word)
    __device__ static __forceinline__ void step_word(uint32_t &z, uint32_t w, const EnvTables &t, uint32_t &s2,
                                                     double &rew, bool &term) {
        if (z >= t.max_steps) { s2 = 0; rew = 0.0; term = true; return; }  // :146-149
        z += 1;
        s2 = w & 511u;
        const uint32_t rc = (w >> 9) & 3u;
        rew = rc == 0 ? -1.0 : (rc == 1 ? -10.0 : 20.0);
        term = (w & (1u << 11)) != 0;
    }
};

// BlackJackEnv (src/env/blackjack.rs): infinite deck, cards 1..=10 uniform.
// z packs the hand: bits 0-7 player sum, 8-15 dealer sum, 16-19 dealer[0],
// bit 20 player_has_ace, bit 21 dealer_has_ace (aces from the first two cards
// only, :54-55).  Dense obs = (p_score*27 + d_score)*2 + p_ace  (p <= 31, d <= 26).
#ifndef RLAMD_BJ_STEP1
#define RLAMD_BJ_STEP1 1   // Blackjack step: hit and stick in one draw loop (EnvDev<BLACKJACK>::step);
                           // cfg 5 0.3511 -> 0.3367 ms per launch (profiles/r05/bj_step1_ab.txt)
#endif
template <> struct EnvDev<RL_ENV_BLACKJACK> {
    static constexpr int A = 2;
    __device__ static __forceinline__ uint32_t score(uint32_t sum, uint32_t ace) {
        return (ace && sum + 10u <= 21u) ? sum + 10u : sum;      // :58-74
    }
    __device__ static __forceinline__ uint32_t obs(uint32_t p, uint32_t d, uint32_t ace) {
        return ((p << 5) + d) * 2u + ace;   // dense index (p*32 + d)*2 + ace: shifts to decode
    }
    __device__ static __forceinline__ uint32_t deal(Rng &r) {    // initialize_hands :47-56
        // two words, four halves: when none is rejected (all but ~4e-4 of deals)
        // they are the deal's four cards; otherwise it is redrawn card by card from
        // the saved state
        const Rng r0 = r;
        const uint32_t w0 = r.next_u32(), w1 = r.next_u32();
        uint32_t p0, p1, d0, d1;
        const bool k0 = card16(w0 >> 16, p0), k1 = card16(w0 & 0xFFFFu, p1), k2 = card16(w1 >> 16, d0),
                   k3 = card16(w1 & 0xFFFFu, d1);
        if (!(k0 && k1 && k2 && k3)) {
            r = r0;
            CardSrc cs;
            p0 = cs.next(r); p1 = cs.next(r); d0 = cs.next(r); d1 = cs.next(r);
        }
        const uint32_t pa = (p0 == 1u || p1 == 1u), da = (d0 == 1u || d1 == 1u);
        return (p0 + p1) | ((d0 + d1) << 8) | (d0 << 16) | (pa << 20) | (da << 21);
    }
    __device__ static __forceinline__ uint32_t reset(uint32_t &z, Rng &r, const EnvTables &) {
        z = deal(r);                                   // :105-116
        const uint32_t pa = (z >> 20) & 1u;
        return obs(score(z & 0xffu, pa), (z >> 16) & 0xfu, pa);
    }
    template <int SLIP = -1, bool AM = false>
    __device__ static __forceinline__ void step(uint32_t &pos, uint32_t &z, uint32_t a, Rng &r,
                                                const EnvTables &, uint32_t &s2, double &rew,
                                                bool &term) {
        uint32_t ps = z & 0xffu, ds = (z >> 8) & 0xffu;
        const uint32_t d0 = (z >> 16) & 0xfu, pa = (z >> 20) & 1u, da = (z >> 21) & 1u;
        if constexpr (RLAMD_BJ_STEP1) {
            // hit and stick in ONE draw loop (a wave holds lanes of both): a hit lane
            // takes the first accepted half of its words (CardSrc), a stick lane the
            // dealer's cards while d < 17, two per word — the draws of the two blocks
            // below, in their order; the wave runs max(words) iterations instead of
            // the hit block and then the dealer loop
            const bool hit = a == 0u;
            uint32_t d = score(ds, da);
            bool act = hit || d < 17u;
            while (act) {
                const uint32_t w = r.next_u32();
                uint32_t c;
                if (card16(w >> 16, c)) {
                    ps += hit ? c : 0u;
                    ds += hit ? 0u : c;
                    d = score(ds, da);
                    act = !hit && d < 17u;
                }
                if (act && card16(w & 0xFFFFu, c)) {
                    ps += hit ? c : 0u;
                    ds += hit ? 0u : c;
                    d = score(ds, da);
                    act = !hit && d < 17u;
                }
            }
            const uint32_t p = score(ps, pa);          // d == score(ds, da) for both kinds
            const bool bust = p > 21u;
            s2 = obs(p, hit ? (bust ? d : d0) : d, pa);
            term = hit ? bust : true;
            rew = hit ? (bust ? -1.0 : 0.0) : (d > 21u ? 1.0 : (p > d ? 1.0 : (p < d ? -1.0 : 0.0)));
            z = ps | (ds << 8) | (z & 0xffff0000u);
            pos = s2;
            return;
        }
        if (a == 0) {                                  // hit :121-138
            CardSrc cs;
            ps += cs.next(r);
            const uint32_t p = score(ps, pa);
            if (p > 21u) {
                s2 = obs(p, score(ds, da), pa); rew = -1.0; term = true;
            } else {
                s2 = obs(p, d0, pa); rew = 0.0; term = false;
            }
        } else {                                       // stick :139-162
            uint32_t d = score(ds, da);
            while (d < 17u) {                          // two cards per word (CardSrc's order)
                const uint32_t w = r.next_u32();
                uint32_t c;
                if (card16(w >> 16, c)) { ds += c; d = score(ds, da); }
                if (d < 17u && card16(w & 0xFFFFu, c)) { ds += c; d = score(ds, da); }
            }
            const uint32_t p = score(ps, pa);
            s2 = obs(p, d, pa);
            term = true;
            rew = d > 21u ? 1.0 : (p > d ? 1.0 : (p < d ? -1.0 : 0.0));
        }
        z = ps | (ds << 8) | (z & 0xffff0000u);
        pos = s2;
    }
    // reset (doR) or step (doS) of one lane in ONE draw loop, for the learner-group
    // kernel where a wave holds lanes of both kinds: a reset lane draws P0, P1, D0,
    // D1, a hit lane one card, a stick lane the dealer's cards while d < 17 — the
    // same draws in the same order as reset() / step(), but the wave runs
    // max(draws) iterations instead of the reset block + the hit block + the
    // dealer loop one after another.
    __device__ static __forceinline__ void advance(bool doR, bool doS, uint32_t &z, uint32_t a, Rng &r,
                                                   uint32_t &s2, double &rew, bool &term) {
        uint32_t ps = z & 0xffu, ds = (z >> 8) & 0xffu, d0 = (z >> 16) & 0xfu, pa = (z >> 20) & 1u,
                 da = (z >> 21) & 1u;
        if (doR) { ps = 0u; ds = 0u; d0 = 0u; pa = 0u; da = 0u; }
        const bool hit = doS && a == 0u, stick = doS && a != 0u;
        const uint32_t nfix = doR ? 4u : (hit ? 1u : 0u);
        CardSrc cs;                                    // the lane's operation draws its own words
        for (uint32_t i = 0;; ++i) {
            if (!(i < nfix || (stick && score(ds, da) < 17u))) break;
            const uint32_t c = cs.next(r);
            if (doR) {
                if (i < 2u) { ps += c; pa |= c == 1u ? 1u : 0u; }
                else { if (i == 2u) d0 = c; ds += c; da |= c == 1u ? 1u : 0u; }
            } else if (hit) {
                ps += c;
            } else {
                ds += c;
            }
        }
        const uint32_t p = score(ps, pa);
        if (doR) {
            z = ps | (ds << 8) | (d0 << 16) | (pa << 20) | (da << 21);
            s2 = obs(p, d0, pa);                       // reset :105-116
        } else if (hit) {                              // :121-138
            if (p > 21u) { s2 = obs(p, score(ds, da), pa); rew = -1.0; term = true; }
            else { s2 = obs(p, d0, pa); rew = 0.0; term = false; }
            z = ps | (ds << 8) | (z & 0xffff0000u);
        } else if (stick) {                            // :139-162
            const uint32_t d = score(ds, da);
            s2 = obs(p, d, pa);
            term = true;
            rew = d > 21u ? 1.0 : (p > d ? 1.0 : (p < d ? -1.0 : 0.0));
            z = ps | (ds << 8) | (z & 0xffff0000u);
        }
    }
};

// ------------------------------------------------------------------ selection helpers
// UniformEpsilonGreed::get_exploration_probs (uniform_epsilon_greed.rs:72-76)
template <int A>
__device__ __forceinline__ void eps_probs(double eps, const double (&q)[A], double (&p)[A]) {
#pragma unroll
    for (int i = 0; i < A; ++i) p[i] = eps / (double)A;
    const uint32_t am = argmax<A>(q);
#pragma unroll
    for (int i = 0; i < A; ++i)
        if ((uint32_t)i == am) p[i] = 1.0 - eps;
}
// sarsa / qlearning / expected_sarsa (src/agent.rs:19-45)
template <int ALGO, int A>
__device__ __forceinline__ double future_q(const double (&q2)[A], uint32_t a2, const double (&p)[A]) {
    if constexpr (ALGO == RL_ALGO_SARSA) return pick<A>(q2, a2);
    else if constexpr (ALGO == RL_ALGO_QLEARNING) return vmax<A>(q2);
    else {
        double f = 0.0;
#pragma unroll
        for (int i = 0; i < A; ++i) f += p[i] * q2[i];
        return f;
    }
}
// decay_epsilon (uniform_epsilon_greed.rs:42-49) with the bins' closure
// new = eps * dm - ds with (dm, ds) = (f, 0) for a*f or (1, d) for a-d: both products
// and differences are exact where the two-branch form is (x*1 = x, x-0 = x), so
// the result is bit-identical without a per-lane select on the decay kind
__device__ __forceinline__ double decay_eps(const KParams &p, double eps) {
    const double nw = eps * p.eps_dm - p.eps_ds;
    return p.eps_final > nw ? eps : nw;
}

// ------------------------------------------------------------------ wave helpers
// set bits of a wave mask below this lane (v_mbcnt_lo + v_mbcnt_hi: two VALU ops,
// where popcount(m & ((1 << lane) - 1)) compiled to two ANDs and two counts)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v |= __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint32_t o = (uint32_t)__shfl_xor((int)v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}

}  // namespace rlamd

// rl_net.h — NeuralPolicy (src/policy/neural_policy.rs) over the 2-layer
// Network of the neural bin (src/bin/frozen_lake_neural.rs:130-134) for the
// private kernel: one lane = one agent with its own parameters, SoA
// [param][lane] in HBM (coalesced: parameter i of a wave's 64 lanes is one
// 512-B row).  Parameter order [W1 n_in x H][b1 H][W2 H x A][b2 A].
//
// Both passes stream over the hidden units j, so no per-lane hidden vector is
// kept: forward accumulates out[i] += act1(z_j) * W2[j][i] in j order (the
// order ndarray's dgemm accumulates in, from 0.0, without FMA — the oracle's
// restatement, oracle/rlref.c net_forward); the backward pass recomputes z_j
// (the same value: W1, b1 are untouched until column j is updated) and
// applies the Dense / Activation backward steps of layers.rs:83-93,135-141
// column by column — W2[j][*] is read (for input_error) before it is written.
//
// Two parameter stores behind one interface (at / w1 / b1 / w2 / b2, n_in, H):
//  - NetLane: the lane's parameters in HBM, any shape and activation (run time);
//  - NetRegs<NIN, H, A, ACT1, ACT2>: the bin's shape as compile-time constants, the
//    lane's parameters held in registers for the whole launch (k_train_private_net:
//    loaded once, written back once; the steps touch no parameter memory).
#pragma once
#include "rl_device.h"

namespace rlamd {

constexpr uint32_t NET_MAX_IN = RL_NET_MAX_INPUT;

struct NetLane {
    static constexpr bool kStatic = false;
    static constexpr int kAct1 = -1, kAct2 = -1;   // run time: KParams::act1 / act2
    double *w;
    uint64_t L, lane;
    uint32_t n_in, H, A;
    __device__ __forceinline__ double &at(uint32_t i) const { return w[(uint64_t)i * L + lane]; }
    __device__ __forceinline__ double &w1(uint32_t k, uint32_t j) const { return at(k * H + j); }
    __device__ __forceinline__ double &b1(uint32_t j) const { return at(n_in * H + j); }
    __device__ __forceinline__ double &w2(uint32_t j, uint32_t i) const { return at(n_in * H + H + j * A + i); }
    __device__ __forceinline__ double &b2(uint32_t i) const { return at(n_in * H + H + H * A + i); }
    template <int AA>
    __device__ __forceinline__ static NetLane make(const KParams &p, uint64_t lane) {
        return NetLane{p.net_w, p.L, lane, p.n_in, p.n_hidden, (uint32_t)AA};
    }
    __device__ __forceinline__ void store(const KParams &, uint64_t) const {}
};

// the lane's parameters in registers (every index below is a compile-time
// constant once the hidden-unit loops are unrolled).  Measured against it on cfg 6
// (one box, alternating): W1 and b1 in LDS with W2 and b2 in registers, 13.2 against
// 10.4 ms per launch — the LDS reads cost more than the registers they free.
template <uint32_t NIN, uint32_t HH, uint32_t AA, int ACT1, int ACT2>
struct NetRegs {
    static constexpr bool kStatic = true;
    static constexpr int kAct1 = ACT1, kAct2 = ACT2;
    static constexpr uint32_t n_in = NIN, H = HH, A = AA, NP = NIN * HH + HH + HH * AA + AA;
    mutable double w[NP];
    __device__ __forceinline__ double &at(uint32_t i) const { return w[i]; }
    __device__ __forceinline__ double &w1(uint32_t k, uint32_t j) const { return w[k * H + j]; }
    __device__ __forceinline__ double &b1(uint32_t j) const { return w[n_in * H + j]; }
    __device__ __forceinline__ double &w2(uint32_t j, uint32_t i) const { return w[n_in * H + H + j * A + i]; }
    __device__ __forceinline__ double &b2(uint32_t i) const { return w[n_in * H + H + H * A + i]; }
    template <int>
    __device__ __forceinline__ static NetRegs make(const KParams &p, uint64_t lane) {
        NetRegs n;
#pragma unroll
        for (uint32_t i = 0; i < NP; ++i) n.w[i] = p.net_w[(uint64_t)i * p.L + lane];
        return n;
    }
    __device__ __forceinline__ void store(const KParams &p, uint64_t lane) const {
        // the base through an empty asm: the store's 196 addresses are computed here,
        // not shared with make()'s loads (kept live across the launch they took 392
        // registers and pushed the parameters into scratch)
        double *b = p.net_w + lane;
        asm volatile("" : "+v"(b));
#pragma unroll
        for (uint32_t i = 0; i < NP; ++i) b[(uint64_t)i * p.L] = w[i];
    }
};
// the bin's network: DenseLayer(1, 32) -> leaky_relu6 -> DenseLayer(32, 4) -> linear
template <uint32_t A>
using NetBin = NetRegs<1, 32, A, RL_ACT_LEAKY_RELU6, RL_ACT_LINEAR>;

template <class NET>
__device__ __forceinline__ double net_act1(const KParams &p, double v) {
    if constexpr (NET::kAct1 >= 0) return act_t<NET::kAct1>(v);
    else return act_f(p.act1, v);
}
template <class NET>
__device__ __forceinline__ double net_act1p(const KParams &p, double v) {
    if constexpr (NET::kAct1 >= 0) return act_pt<NET::kAct1>(v);
    else return act_fp(p.act1, v);
}
template <class NET>
__device__ __forceinline__ int net_act2(const KParams &p) {
    if constexpr (NET::kAct2 >= 0) return NET::kAct2;
    else return p.act2;
}
// f(j) for every hidden unit j in order (unrolled when the shape is static)
template <class NET, class F>
__device__ __forceinline__ void for_hidden(const NET &n, F &&f) {
    if constexpr (NET::kStatic) {
#pragma unroll
        for (uint32_t j = 0; j < NET::H; ++j) f(j);
    } else {
        for (uint32_t j = 0; j < n.H; ++j) f(j);
    }
}

// input-adapter features of state s into registers
__device__ __forceinline__ void net_input(const KParams &p, uint32_t s, double (&x)[NET_MAX_IN]) {
#pragma unroll
    for (uint32_t k = 0; k < NET_MAX_IN; ++k) x[k] = k < p.n_in ? p.feat[s * p.n_in + k] : 0.0;
}

// z_j = (0.0 + sum_k x_k W1[k][j]) + b1[j]  (DenseLayer::forward_propagation, layers.rs:78-81)
template <class NET>
__device__ __forceinline__ double net_z(const NET &n, const double (&x)[NET_MAX_IN], uint32_t j) {
    double z = 0.0;
#pragma unroll
    for (uint32_t k = 0; k < NET_MAX_IN; ++k)
        if (k < n.n_in) z = z + x[k] * n.w1(k, j);
    return z + n.b1(j);
}

template <int A, class NET>
__device__ __forceinline__ void net_output(const KParams &p, const double (&opre)[A], double (&y)[A]);

// Network::predict (src/network.rs:51-58): opre = pre-activation output, y = act2(opre)
template <int A, class NET>
__device__ __forceinline__ void net_forward(const KParams &p, const NET &n, const double (&x)[NET_MAX_IN],
                                            double (&opre)[A], double (&y)[A]) {
    double acc[A];
#pragma unroll
    for (int i = 0; i < A; ++i) acc[i] = 0.0;
    for_hidden(n, [&](uint32_t j) {
        const double h = net_act1<NET>(p, net_z(n, x, j));
#pragma unroll
        for (int i = 0; i < A; ++i) acc[i] = acc[i] + h * n.w2(j, (uint32_t)i);
    });
#pragma unroll
    for (int i = 0; i < A; ++i) opre[i] = acc[i] + n.b2((uint32_t)i);
    net_output<A, NET>(p, opre, y);
}

// the output layer's activation: y = act2(opre)
template <int A, class NET>
__device__ __forceinline__ void net_output(const KParams &p, const double (&opre)[A], double (&y)[A]) {
    const int act2 = net_act2<NET>(p);
    if (act2 == RL_ACT_SOFTMAX) {          // activation.rs:64-68, ndarray_max utils.rs:23-31
        double m = opre[0], e[A], sum = 0.0;
#pragma unroll
        for (int i = 1; i < A; ++i) m = opre[i] > m ? opre[i] : m;
#pragma unroll
        for (int i = 0; i < A; ++i) { e[i] = rl_exp(opre[i] - m); sum = sum + e[i]; }
#pragma unroll
        for (int i = 0; i < A; ++i) y[i] = e[i] / sum;
    } else if constexpr (NET::kAct2 >= 0) {
#pragma unroll
        for (int i = 0; i < A; ++i) y[i] = act_t<NET::kAct2>(opre[i]);
    } else {
#pragma unroll
        for (int i = 0; i < A; ++i) y[i] = act_f(act2, opre[i]);
    }
}

// two predicts with the same parameters in one pass over the hidden units (the
// step's get_action(s') and update's get_values(s)): every chain's operations in
// the forward's own order, so each result is the forward's; each parameter is read
// once for both, and the two chains are independent work for the same issue slots
template <int A, class NET>
__device__ __forceinline__ void net_forward2(const KParams &p, const NET &n, const double (&xa)[NET_MAX_IN],
                                             const double (&xb)[NET_MAX_IN], double (&oa)[A], double (&ya)[A],
                                             double (&ob)[A], double (&yb)[A]) {
    double acc_a[A], acc_b[A];
#pragma unroll
    for (int i = 0; i < A; ++i) { acc_a[i] = 0.0; acc_b[i] = 0.0; }
    for_hidden(n, [&](uint32_t j) {
        const double ha = net_act1<NET>(p, net_z(n, xa, j));
        const double hb = net_act1<NET>(p, net_z(n, xb, j));
#pragma unroll
        for (int i = 0; i < A; ++i) {
            const double w = n.w2(j, (uint32_t)i);
            acc_a[i] = acc_a[i] + ha * w;
            acc_b[i] = acc_b[i] + hb * w;
        }
    });
#pragma unroll
    for (int i = 0; i < A; ++i) { oa[i] = acc_a[i] + n.b2((uint32_t)i); ob[i] = acc_b[i] + n.b2((uint32_t)i); }
    net_output<A, NET>(p, oa, ya);
    net_output<A, NET>(p, ob, yb);
}

// Network::fit (src/network.rs:61-80) at input x, given that forward pass
// (opre, y) and the target t: mse_prime (loss.rs:4-9), then the layers backward.
template <int A, class NET>
__device__ __forceinline__ void net_fit(const KParams &p, const NET &n, const double (&x)[NET_MAX_IN],
                                        const double (&opre)[A], const double (&y)[A], const double (&t)[A]) {
    const double lr = p.lr;
    const int act2 = net_act2<NET>(p);
    double e2[A];
#pragma unroll
    for (int i = 0; i < A; ++i) {
        // softmax_prime == softmax (activation.rs:70-74): the forward's y
        double pr;
        if constexpr (NET::kAct2 >= 0 && NET::kAct2 != RL_ACT_SOFTMAX) pr = act_pt<NET::kAct2>(opre[i]);
        else pr = act2 == RL_ACT_SOFTMAX ? y[i] : act_fp(act2, opre[i]);
        e2[i] = pr * ((2.0 * (y[i] - t[i])) / (double)A);
    }
    for_hidden(n, [&](uint32_t j) {
        const double z = net_z(n, x, j);
        const double h = net_act1<NET>(p, z);
        double ie = 0.0;                     // input_error = e2.dot(W2.t()), old W2
#pragma unroll
        for (int i = 0; i < A; ++i) ie = ie + e2[i] * n.w2(j, (uint32_t)i);
#pragma unroll
        for (int i = 0; i < A; ++i) {        // W2 -= lr * h.t().dot(e2)
            double &wv = n.w2(j, (uint32_t)i);
            wv = wv - lr * (0.0 + h * e2[i]);
        }
        const double e1 = net_act1p<NET>(p, z) * ie;
#pragma unroll
        for (uint32_t k = 0; k < NET_MAX_IN; ++k) {
            if (k < n.n_in) {                // W1 -= lr * x.t().dot(e1)
                double &wv = n.w1(k, j);
                wv = wv - lr * (0.0 + x[k] * e1);
            }
        }
        double &bv = n.b1(j);
        bv = bv - lr * e1;
    });
#pragma unroll
    for (int i = 0; i < A; ++i) {
        double &bv = n.b2((uint32_t)i);
        bv = bv - lr * e2[i];
    }
}

// get_values with a one-entry cache: the forward at the state last evaluated is
// reused until the parameters change (get_action(s') then update's
// get_values(s'), and update's get_values(s) then Policy::update's) — the
// same numbers the reference recomputes.
template <int A>
struct NetCache {
    uint32_t s = 0xffffffffu;
    double opre[A], y[A];
    template <class NET>
    __device__ __forceinline__ void get(const KParams &p, const NET &n, uint32_t st) {
        if (st == s) return;
        double x[NET_MAX_IN];
        net_input(p, st, x);
        net_forward<A>(p, n, x, opre, y);
        s = st;
    }
    __device__ __forceinline__ void invalidate() { s = 0xffffffffu; }
    // o's entry when it holds st and this one does not (element-wise selects:
    // the entries stay in registers)
    __device__ __forceinline__ void take(const NetCache &o, uint32_t st) {
        const bool t = s != st && o.s == st;
#pragma unroll
        for (int i = 0; i < A; ++i) { opre[i] = t ? o.opre[i] : opre[i]; y[i] = t ? o.y[i] : y[i]; }
        s = t ? st : s;
    }
    // this entry := predict(sa), o := predict(sb), in one pass (net_forward2)
    template <class NET>
    __device__ __forceinline__ void get_pair(const KParams &p, const NET &n, uint32_t sa, NetCache &o, uint32_t sb) {
        double xa[NET_MAX_IN], xb[NET_MAX_IN];
        net_input(p, sa, xa);
        net_input(p, sb, xb);
        net_forward2<A>(p, n, xa, xb, opre, y, o.opre, o.y);
        s = sa;
        o.s = sb;
    }
};

// NeuralPolicy::update (neural_policy.rs:55-62): y = get_values(s), y[a] += x, fit
template <int A, class NET>
__device__ __forceinline__ void net_policy_update(const KParams &p, const NET &n, NetCache<A> &c, uint32_t s,
                                                  uint32_t a, double xv) {
    c.get(p, n, s);
    double t[A];
#pragma unroll
    for (int i = 0; i < A; ++i) t[i] = (uint32_t)i == a ? c.y[i] + xv : c.y[i];
    double x[NET_MAX_IN];
    net_input(p, s, x);
    net_fit<A>(p, n, x, c.opre, c.y, t);
    c.invalidate();
}

}  // namespace rlamd

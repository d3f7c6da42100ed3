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
#pragma once
#include "rl_device.h"

namespace rlamd {

constexpr uint32_t NET_MAX_IN = RL_NET_MAX_INPUT;

struct NetLane {
    double *w;
    uint64_t L, lane;
    uint32_t n_in, H, A;
    __device__ __forceinline__ double &at(uint32_t i) const { return w[(uint64_t)i * L + lane]; }
    __device__ __forceinline__ double &w1(uint32_t k, uint32_t j) const { return at(k * H + j); }
    __device__ __forceinline__ double &b1(uint32_t j) const { return at(n_in * H + j); }
    __device__ __forceinline__ double &w2(uint32_t j, uint32_t i) const { return at(n_in * H + H + j * A + i); }
    __device__ __forceinline__ double &b2(uint32_t i) const { return at(n_in * H + H + H * A + i); }
};

// input-adapter features of state s into registers
__device__ __forceinline__ void net_input(const KParams &p, uint32_t s, double (&x)[NET_MAX_IN]) {
#pragma unroll
    for (uint32_t k = 0; k < NET_MAX_IN; ++k) x[k] = k < p.n_in ? p.feat[s * p.n_in + k] : 0.0;
}

// z_j = (0.0 + sum_k x_k W1[k][j]) + b1[j]  (DenseLayer::forward_propagation, layers.rs:78-81)
__device__ __forceinline__ double net_z(const NetLane &n, const double (&x)[NET_MAX_IN], uint32_t j) {
    double z = 0.0;
#pragma unroll
    for (uint32_t k = 0; k < NET_MAX_IN; ++k)
        if (k < n.n_in) z = z + x[k] * n.w1(k, j);
    return z + n.b1(j);
}

// Network::predict (src/network.rs:51-58): opre = pre-activation output, y = act2(opre)
template <int A>
__device__ __forceinline__ void net_forward(const KParams &p, const NetLane &n, const double (&x)[NET_MAX_IN],
                                            double (&opre)[A], double (&y)[A]) {
    double acc[A];
#pragma unroll
    for (int i = 0; i < A; ++i) acc[i] = 0.0;
    for (uint32_t j = 0; j < n.H; ++j) {
        const double h = act_f(p.act1, net_z(n, x, j));
#pragma unroll
        for (int i = 0; i < A; ++i) acc[i] = acc[i] + h * n.w2(j, (uint32_t)i);
    }
#pragma unroll
    for (int i = 0; i < A; ++i) opre[i] = acc[i] + n.b2((uint32_t)i);
    if (p.act2 == RL_ACT_SOFTMAX) {          // activation.rs:64-68, ndarray_max utils.rs:23-31
        double m = opre[0], e[A], sum = 0.0;
#pragma unroll
        for (int i = 1; i < A; ++i) m = opre[i] > m ? opre[i] : m;
#pragma unroll
        for (int i = 0; i < A; ++i) { e[i] = rl_exp(opre[i] - m); sum = sum + e[i]; }
#pragma unroll
        for (int i = 0; i < A; ++i) y[i] = e[i] / sum;
    } else {
#pragma unroll
        for (int i = 0; i < A; ++i) y[i] = act_f(p.act2, opre[i]);
    }
}

// Network::fit (src/network.rs:61-80) at input x, given that forward pass
// (opre, y) and the target t: mse_prime (loss.rs:4-9), then the layers backward.
template <int A>
__device__ __forceinline__ void net_fit(const KParams &p, const NetLane &n, const double (&x)[NET_MAX_IN],
                                        const double (&opre)[A], const double (&y)[A], const double (&t)[A]) {
    const double lr = p.lr;
    double e2[A];
#pragma unroll
    for (int i = 0; i < A; ++i) {
        // softmax_prime == softmax (activation.rs:70-74): the forward's y
        const double pr = p.act2 == RL_ACT_SOFTMAX ? y[i] : act_fp(p.act2, opre[i]);
        e2[i] = pr * ((2.0 * (y[i] - t[i])) / (double)A);
    }
    for (uint32_t j = 0; j < n.H; ++j) {
        const double z = net_z(n, x, j);
        const double h = act_f(p.act1, z);
        double ie = 0.0;                     // input_error = e2.dot(W2.t()), old W2
#pragma unroll
        for (int i = 0; i < A; ++i) ie = ie + e2[i] * n.w2(j, (uint32_t)i);
#pragma unroll
        for (int i = 0; i < A; ++i) {        // W2 -= lr * h.t().dot(e2)
            double &wv = n.w2(j, (uint32_t)i);
            wv = wv - lr * (0.0 + h * e2[i]);
        }
        const double e1 = act_fp(p.act1, z) * ie;
#pragma unroll
        for (uint32_t k = 0; k < NET_MAX_IN; ++k) {
            if (k < n.n_in) {                // W1 -= lr * x.t().dot(e1)
                double &wv = n.w1(k, j);
                wv = wv - lr * (0.0 + x[k] * e1);
            }
        }
        double &bv = n.b1(j);
        bv = bv - lr * e1;
    }
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
    __device__ __forceinline__ void get(const KParams &p, const NetLane &n, uint32_t st) {
        if (st == s) return;
        double x[NET_MAX_IN];
        net_input(p, st, x);
        net_forward<A>(p, n, x, opre, y);
        s = st;
    }
    __device__ __forceinline__ void invalidate() { s = 0xffffffffu; }
};

// NeuralPolicy::update (neural_policy.rs:55-62): y = get_values(s), y[a] += x, fit
template <int A>
__device__ __forceinline__ void net_policy_update(const KParams &p, const NetLane &n, NetCache<A> &c, uint32_t s,
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

// rl_taxi.h — TaxiEnv's dynamics as arithmetic, shared by the gfx950 kernels
// (rl_device.h EnvDev<RL_ENV_TAXI>) and the host runtime, which checks them
// against the table it builds from TaxiEnv::new's loop (rl_host.cpp build_env).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace rlamd {

struct TaxiMap {
    // MAP[1+row][2*col+2] == ':' (RIGHT passes), bit row*5+col (taxi.rs:22-30, :85-92)
    static constexpr uint32_t right_ok() {
        const char *m[5] = {"|R: | : :G|", "| : | : : |", "| : : : : |", "| | : | : |", "|Y| : |B: |"};
        uint32_t k = 0;
        for (int r = 0; r < 5; ++r)
            for (int c = 0; c < 5; ++c)
                if (m[r][2 * c + 2] == ':') k |= 1u << (r * 5 + c);
        return k;
    }
    // LEFT passes iff MAP[1+row][2*col] == ':', the same character as RIGHT from col-1
    static constexpr uint32_t left_ok() { return (right_ok() << 1) & ~0x108421u; }   // no wrap into col 0
    static constexpr uint32_t locs = 0u | (4u << 8) | (20u << 16) | (23u << 24);        // LOCS cells (taxi.rs:31)
};
__host__ __device__ inline uint32_t taxi_word(uint32_t s, uint32_t a) {
    constexpr uint32_t RIGHT = TaxiMap::right_ok(), LEFT = TaxiMap::left_ok();
    const uint32_t dest = s & 3u, q = s >> 2, pass = q % 5u, cell = q / 5u, row = cell / 5u, col = cell - row * 5u;
    uint32_t nr = row, nc = col, np = pass, rc = 0u, term = 0u;
    if (a == 0u) nr = row < 4u ? row + 1u : 4u;
    else if (a == 1u) nr = row > 0u ? row - 1u : 0u;
    else if (a == 2u) nc = (RIGHT >> cell) & 1u ? col + 1u : col;
    else if (a == 3u) nc = (LEFT >> cell) & 1u ? col - 1u : col;
    else if (a == 4u) {                                    // pickup
        if (pass < 4u && cell == ((TaxiMap::locs >> (8u * pass)) & 0xffu)) np = 4u;
        else rc = 1u;
    } else {                                               // dropoff
        if (pass == 4u && cell == ((TaxiMap::locs >> (8u * dest)) & 0xffu)) { np = dest; term = 1u; rc = 2u; }
        else rc = 1u;
    }
    return (((nr * 5u + nc) * 5u + np) * 4u + dest) | (rc << 9) | (term << 11);
}
// Env::reset's categorical_sample over the start distribution (taxi.rs:136-137,
// utils.rs:33-43): the 300 states with pass < 4 && pass != dest carry 1/300 each,
// in encode order; c_k = the running sum after the k-th of them (cdf[state(k)]).
// The answer is the first k with c_k > u (else state 0, u >= c_300 =
// 0.9999999999999961).  c_k = k/300 within 1e-13 while the c_k are 1/300 apart,
// so k is one of floor(u*300) .. floor(u*300)+2: three probes of the HBM cdf
// instead of a 500-entry LDS table (build_env checks every boundary).  The three
// loads are independent (issued together: one memory latency, not three) and
// the first probe whose c_k > u wins, as a scan would find it.
__host__ __device__ inline uint32_t taxi_start_state(uint32_t k) {   // k = 1..300
    const uint32_t k0 = k - 1u, cell = k0 / 12u, j = k0 - cell * 12u, pass = j / 3u, r3 = j - pass * 3u;
    return cell * 20u + pass * 4u + r3 + (r3 >= pass ? 1u : 0u);
}
__host__ __device__ inline uint32_t taxi_start(const double *cdf, double u) {
    const uint32_t g = (uint32_t)(u * 300.0);
    const uint32_t k = g < 1u ? 1u : g;                    // <= 300: u < 1
    const uint32_t s0 = taxi_start_state(k);
    const uint32_t s1 = k + 1u <= 300u ? taxi_start_state(k + 1u) : s0;
    const uint32_t s2 = k + 2u <= 300u ? taxi_start_state(k + 2u) : s0;
    const double c0 = cdf[s0], c1 = cdf[s1], c2 = cdf[s2];
    if (c0 > u) return s0;
    if (k + 1u <= 300u && c1 > u) return s1;
    if (k + 2u <= 300u && c2 > u) return s2;
    return 0u;
}

}  // namespace rlamd

// lds_gather.hip — LDS bank-conflict floor of random row gathers on gfx950
// (the read pattern of cfg 5's Q rows: every lane of a wave reads the row of its
// own, independent state).  Each kernel reads ROWS-row tables from LDS at
// per-lane pseudo-random rows, N reads per thread; rocprofv3 --pmc
// SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE per dispatch gives the conflict share.
//   k_rand_b128   16-B rows (one ds_read_b128), uniform over 484 rows
//   k_rand_b64    8-B rows (ds_read_b64), uniform over 968 rows (same bytes)
//   k_rand_b128x2 32-B rows read as two ds_read_b128 (both tables of a row)
//   k_seq_b128    lane i reads row i (conflict-free control)
//   k_bcast_b128  every lane of a wave reads the same row (broadcast control)
//   k_atom_rand   ds_add_u64 (no return) to a random one of 192 entries (cfg 4's
//                 pair table: the trace sweep's contributions)
//   k_atom_same   ds_add_u64, every lane of a wave to one entry
//   k_atom_lane   ds_add_u64, lane i to entry i (distinct, conflict-free)
// build: hipcc --offload-arch=gfx950 -O3 scripts/lds_gather.hip -o rl-rust_amd/exp/lds_gather
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int ROWS = 484;   // Blackjack's reachable rows (bj_row)
constexpr int N = 256;      // reads per thread

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t row_of(uint32_t t, uint32_t it, uint32_t rows) {
    return __umulhi(mix(t * 0x9E3779B9u + it * 0x85EBCA6Bu + 1u), rows);
}

template <int KIND>
__global__ void __launch_bounds__(256) k_gather(double *out) {
    __shared__ double2 T[2 * ROWS];
    for (int i = threadIdx.x; i < 2 * ROWS; i += blockDim.x) T[i] = make_double2(i, 2 * i);
    __syncthreads();
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    double acc = 0.0;
    for (uint32_t it = 0; it < N; ++it) {
        if constexpr (KIND == 0) {            // random 16-B rows
            const double2 v = T[row_of(t, it, ROWS)];
            acc += v.x + v.y;
        } else if constexpr (KIND == 1) {     // random 8-B rows over the same bytes
            const double v = ((const double *)T)[row_of(t, it, 2 * ROWS)];
            acc += v;
        } else if constexpr (KIND == 2) {     // random 32-B rows: two 16-B reads
            const uint32_t r = row_of(t, it, ROWS);
            const double2 a = T[2 * r], b = T[2 * r + 1];
            acc += a.x + a.y + b.x + b.y;
        } else if constexpr (KIND == 3) {     // lane i: row i (+ it): conflict-free
            const double2 v = T[((threadIdx.x & 63u) + it) % ROWS];
            acc += v.x + v.y;
        } else if constexpr (KIND == 4) {     // one row per wave: broadcast
            const uint32_t w = __builtin_amdgcn_readfirstlane(row_of(t >> 6, it, ROWS));
            const double2 v = T[w];
            acc += v.x + v.y;
        } else {                              // 64-bit LDS atomics (no return)
            unsigned long long *U = (unsigned long long *)T;
            const uint32_t i = KIND == 5 ? row_of(t, it, 192u)
                             : KIND == 6 ? __builtin_amdgcn_readfirstlane(row_of(t >> 6, it, 192u))
                                         : (threadIdx.x & 63u) * 3u;
            atomicAdd(&U[i], (unsigned long long)(it + 1u));
        }
    }
    if constexpr (KIND >= 5) {
        __syncthreads();
        acc = (double)((unsigned long long *)T)[threadIdx.x % 192u];
    }
    out[t] = acc;
}

int main() {
    const int blocks = 2048, threads = 256;
    double *out;
    if (hipMalloc(&out, sizeof(double) * blocks * threads) != hipSuccess) return 1;
    const char *names[] = {"rand_b128", "rand_b64", "rand_b128x2", "seq_b128", "bcast_b128",
                           "atom_rand192", "atom_same", "atom_lane"};
    k_gather<3><<<blocks, threads>>>(out);   // warm-up dispatch (module load, clocks)
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    for (int k = 0; k < 8; ++k) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0);
        switch (k) {
            case 0: k_gather<0><<<blocks, threads>>>(out); break;
            case 1: k_gather<1><<<blocks, threads>>>(out); break;
            case 2: k_gather<2><<<blocks, threads>>>(out); break;
            case 3: k_gather<3><<<blocks, threads>>>(out); break;
            case 4: k_gather<4><<<blocks, threads>>>(out); break;
            case 5: k_gather<5><<<blocks, threads>>>(out); break;
            case 6: k_gather<6><<<blocks, threads>>>(out); break;
            default: k_gather<7><<<blocks, threads>>>(out); break;
        }
        (void)hipEventRecord(e1);
        if (hipEventSynchronize(e1) != hipSuccess) return 2;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("{\"kernel\": \"%s\", \"ms\": %.4f}\n", names[k], ms);
    }
    (void)hipFree(out);
    return 0;
}

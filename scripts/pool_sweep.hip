// pool_sweep.hip — cfg 4's pair-pool sweep alone, at cfg 4's occupancy, replaying
// the real workload ("measure the sweep's LDS atomic and read
// pattern in isolation ... and state the floor it implies per env-step").
//
// Input: what the training kernel knows about each lane after its env step and
// selection, recorded from the real agent by scripts/cfg4_sweep_floor.py: one u16
// per (launch, step, lane) = pair id s*4+a (bits 0-7) | trains (8) | episode ends
// (9).  Per step, exactly as k_train_shared's pool path (rl_train_impl.h, POOL with
// RLAMD_POOL_LREC, U = RLAMD_SWEEP_U = 4; elegibility_traces_agent.rs:75-101):
//   - the lane's visited-pair bits decide hit (E += 1 inside the sweep) or new pair
//     (contributes after the sweep, joins the pool unless its episode ends);
//   - the lane writes its 16-byte {td, pk} record; the wave sweeps its pool 64
//     items per round (tag u16 + E f64 from LDS, the item's lane record, the SUM
//     atomic on the step grid, the row count for a first-of-state item) and writes
//     the kept items back compacted (ballot + mbcnt);
//   - then the group's contributions barrier and a settle stand-in (threads read
//     and zero SUM / CNTR) behind a second barrier.
// Not here: the env step, the selection, the TD, the grid's code pass, Q.  td is a
// fixed function of the input (finite); the grid exponent is fixed.
// SWEEP=0 builds the same kernel without the item loop (the per-step remainder);
// UU / PF: sweep width and next-round prefetch variants (the checksum of the SUM /
// CNTR settles must agree between the sweep variants).
//
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/pool_sweep.hip -o rl-rust_amd/exp/pool_sweep
//   run:   pool_sweep <steps.u16> <lanes> <steps_per_launch> <launches> [tile]
//          (prints one JSON line per launch and variant; tile T replays the input
//          lanes T times over T x lanes: the same pattern at T times the groups)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

constexpr uint32_t A = 4, S = 48, SA = S * A, G = 256, NW = G / 64, U = 4;
constexpr uint32_t CAP = 40u * 1024u / (NW * 10u);     // trc_kb 40: 1024 items per wave (smem_layout)
constexpr int PBW = 6;                                 // 192 pair ids

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(2); } } while (0)

__device__ __forceinline__ uint32_t opq(uint32_t x) { asm volatile("" : "+v"(x)); return x; }
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

struct Lds {
    unsigned long long sum[SA];
    uint32_t cntr[S];
    uint4 lr[NW][64];
    uint16_t pt[NW][CAP];
    double pe[NW][CAP];
};

template <int SWEEP, int UU = U, int PF = 0>
__global__ void __launch_bounds__(G) k_sweep(const uint16_t *__restrict__ in, uint32_t L, uint32_t LI, uint32_t K,
                                             uint16_t *HT, double *HE, uint32_t *HN, uint32_t *PB,
                                             unsigned long long *out, uint32_t *ovf) {
    __shared__ Lds sm;
    const uint32_t tid = threadIdx.x, plid = tid & 63u, w = tid >> 6;
    const uint32_t lane = blockIdx.x * G + tid, wg = blockIdx.x * NW + w;
    uint16_t *PT = sm.pt[w];
    double *PE = sm.pe[w];
    uint4 *LR = sm.lr[w];
    uint32_t npool = HN[wg];
    for (uint32_t q = plid; q < npool; q += 64u) { PT[q] = HT[(size_t)wg * CAP + q]; PE[q] = HE[(size_t)wg * CAP + q]; }
    uint32_t pbits[PBW];
#pragma unroll
    for (int i = 0; i < PBW; ++i) pbits[i] = PB[(size_t)lane * PBW + i];
    for (uint32_t i = tid; i < SA; i += G) sm.sum[i] = 0ull;
    for (uint32_t i = tid; i < S; i += G) sm.cntr[i] = 0u;
    __syncthreads();
    const double lr = 0.1, gl = 0.9 * 0.5;   // gamma * lambda
    const int e_tr = -40;
    unsigned long long acc = 0ull;
    uint32_t over = 0u;
    const uint32_t il = lane % LI;           // tiled runs: lane i replays input lane i mod LI
    uint32_t x = in[il];
    for (uint32_t k = 0; k < K; ++k) {
        const uint32_t xn = k + 1u < K ? in[(size_t)(k + 1u) * LI + il] : 0u;   // next step's input, early
        const bool train = (x >> 8) & 1u, term = (x >> 9) & 1u;
        const double td = (double)(int)((x * 2654435761u) >> 12) * 0x1p-20 - 0.5;
        uint32_t hid = 0x1ffu, nid = 0u;
        bool newp = false, first_new = false;
        if (train) {
            const uint32_t id = x & 0xffu;
            uint32_t wd = opq(pbits[0]);
#pragma unroll
            for (int i = 1; i < PBW; ++i) wd = (id >> 5) == (uint32_t)i ? opq(pbits[i]) : wd;
            if ((wd >> (id & 31u)) & 1u) {
                hid = id;
            } else {
                newp = true;
                nid = id;
                first_new = ((wd >> ((id & ~3u) & 31u)) & 0xfu) == 0u;
#pragma unroll
                for (int i = 0; i < PBW; ++i) pbits[i] |= (id >> 5) == (uint32_t)i ? (1u << (id & 31u)) : 0u;
            }
        }
        const uint32_t pk = hid | (train ? 1u << 20 : 0u) | (train && term ? 1u << 21 : 0u);
        const uint64_t tb = (uint64_t)__double_as_longlong(td);
        LR[plid] = make_uint4((uint32_t)tb, (uint32_t)(tb >> 32), pk, 0u);
        __builtin_amdgcn_wave_barrier();
        uint32_t wpos = 0;
        if constexpr (SWEEP) {
            // PF: the next round's tags and E read before this round's atomics and
            // write-back (compaction only moves items down: every position this
            // round writes is below the next round's first item)
            uint32_t tgn[UU];
            double evn[UU];
            if constexpr (PF) {
#pragma unroll
                for (uint32_t u = 0; u < UU; ++u) {
                    const uint32_t q = 64u * u + plid;
                    tgn[u] = PT[q < npool ? q : 0u];
                    evn[u] = PE[q < npool ? q : 0u];
                }
            }
            for (uint32_t q0 = 0; q0 < npool; q0 += 64u * UU) {
                uint32_t tg[UU], pkv[UU];
                double ev[UU], tdv[UU];
#pragma unroll
                for (uint32_t u = 0; u < UU; ++u) {
                    const uint32_t q = q0 + 64u * u + plid;
                    if constexpr (PF) {
                        tg[u] = tgn[u];
                        ev[u] = evn[u];
                    } else {
                        tg[u] = PT[q < npool ? q : 0u];
                        ev[u] = PE[q < npool ? q : 0u];
                    }
                }
                if constexpr (PF) {
                    if (q0 + 64u * UU < npool) {
#pragma unroll
                        for (uint32_t u = 0; u < UU; ++u) {
                            const uint32_t q = q0 + 64u * (UU + u) + plid;
                            tgn[u] = PT[q < npool ? q : 0u];
                            evn[u] = PE[q < npool ? q : 0u];
                        }
                    }
                }
#pragma unroll
                for (uint32_t u = 0; u < UU; ++u) {
                    const uint4 r = LR[(tg[u] >> 8) & 63u];
                    tdv[u] = __longlong_as_double((long long)(((uint64_t)r.y << 32) | r.x));
                    pkv[u] = r.z;
                }
#pragma unroll
                for (uint32_t u = 0; u < UU; ++u) {
                    const uint32_t q = q0 + 64u * u + plid;
                    const bool valid = q < npool;
                    const bool istr = valid && ((pkv[u] >> 20) & 1u);
                    const bool keep = valid && !((pkv[u] >> 21) & 1u);
                    double en = ev[u];
                    if (istr) {
                        const uint32_t id = tg[u] & 0xffu;
                        const double e1 = id == (pkv[u] & 0x1ffu) ? ev[u] + 1.0 : ev[u];
                        if (tg[u] & 0x8000u) atomicAdd(&sm.cntr[id >> 2], 1u);
                        const double d = lr * (tdv[u] * e1);
                        const double y = __builtin_ldexp(d, -e_tr) + 0x1.8p52;
                        const int64_t raw = (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull);
                        if (raw) atomicAdd(&sm.sum[id], (unsigned long long)raw);
                        en = e1 * gl;
                    }
                    const uint64_t m = __ballot(keep);
                    const uint32_t pos = wpos + lanes_below(m);
                    if (keep) { PT[pos] = (uint16_t)tg[u]; PE[pos] = en; }
                    wpos += (uint32_t)__popcll(m);
                }
            }
        } else {
            // no item loop: the pool keeps its size (the kept count is still formed)
            wpos = npool;
        }
        if (newp) {
            if (first_new) atomicAdd(&sm.cntr[nid >> 2], 1u);
            const double y = __builtin_ldexp(lr * td, -e_tr) + 0x1.8p52;
            const int64_t raw = (int64_t)((uint64_t)__double_as_longlong(y) - 0x4338000000000000ull);
            if (raw) atomicAdd(&sm.sum[nid], (unsigned long long)raw);
        }
        const bool keepn = newp && !term;
        const uint64_t m = __ballot(keepn);
        if (keepn) {
            const uint32_t pos = wpos + lanes_below(m);
            const uint16_t tag = (uint16_t)(nid | (plid << 8) | (first_new ? 0x8000u : 0u));
            if (pos < CAP) { PT[pos] = tag; PE[pos] = gl; }
        }
        npool = wpos + (uint32_t)__popcll(m);
        if (npool > CAP) { over += npool - CAP; npool = CAP; }
        if (train && term) {
#pragma unroll
            for (int i = 0; i < PBW; ++i) pbits[i] = 0u;
        }
        __syncthreads();                       // the step's contributions are in
        for (uint32_t i = tid; i < SA; i += G) { acc += sm.sum[i]; sm.sum[i] = 0ull; }   // settle stand-in
        for (uint32_t i = tid; i < S; i += G) { acc += sm.cntr[i]; sm.cntr[i] = 0u; }
        __syncthreads();
        x = xn;
    }
    for (uint32_t q = plid; q < npool; q += 64u) { HT[(size_t)wg * CAP + q] = PT[q]; HE[(size_t)wg * CAP + q] = PE[q]; }
    if (plid == 0) HN[wg] = npool;
#pragma unroll
    for (int i = 0; i < PBW; ++i) PB[(size_t)lane * PBW + i] = pbits[i];
    out[lane] += acc;
    if (plid == 0 && over) atomicAdd(ovf, over);
}

int main(int argc, char **argv) {
    if (argc < 5) { fprintf(stderr, "usage: %s steps.u16 lanes steps_per_launch launches\n", argv[0]); return 1; }
    const uint32_t LI = (uint32_t)atoi(argv[2]), K = (uint32_t)atoi(argv[3]), NL = (uint32_t)atoi(argv[4]);
    const uint32_t T = argc > 5 ? (uint32_t)atoi(argv[5]) : 1u, L = LI * T;
    if (L % G != 0 || K == 0 || NL == 0) { fprintf(stderr, "lanes must be a multiple of %u\n", G); return 1; }
    const size_t per = (size_t)K * LI, n = per * NL;
    std::vector<uint16_t> h(n);
    FILE *f = fopen(argv[1], "rb");
    if (!f || fread(h.data(), 2, n, f) != n) { fprintf(stderr, "short input %s\n", argv[1]); return 1; }
    fclose(f);
    const uint32_t waves = L / 64u, blocks = L / G;
    uint16_t *in, *HT; double *HE; uint32_t *HN, *PB, *ovf; unsigned long long *out;
    CK(hipMalloc(&in, n * 2));
    CK(hipMemcpy(in, h.data(), n * 2, hipMemcpyHostToDevice));
    CK(hipMalloc(&HT, (size_t)waves * CAP * 2));
    CK(hipMalloc(&HE, (size_t)waves * CAP * 8));
    CK(hipMalloc(&HN, (size_t)waves * 4));
    CK(hipMalloc(&PB, (size_t)L * PBW * 4));
    CK(hipMalloc(&out, (size_t)L * 8));
    CK(hipMalloc(&ovf, 4));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // variants: 0 the library's sweep (U 4), 1 no item loop, 2 U 4 + next-round
    // prefetch, 3 U 8, 4 U 2 + prefetch
    const char *vname[] = {"sweep", "no_sweep", "sweep_pf", "sweep_u8", "sweep_u2_pf"};
    for (int v = 0; v < 5; ++v) {
        CK(hipMemset(HN, 0, (size_t)waves * 4));
        CK(hipMemset(PB, 0, (size_t)L * PBW * 4));
        CK(hipMemset(out, 0, (size_t)L * 8));
        for (uint32_t l = 0; l < NL; ++l) {
            CK(hipMemset(ovf, 0, 4));
            CK(hipEventRecord(e0));
            const uint16_t *il = in + l * per;
            switch (v) {
                case 0: k_sweep<1><<<blocks, G>>>(il, L, LI, K, HT, HE, HN, PB, out, ovf); break;
                case 1: k_sweep<0><<<blocks, G>>>(il, L, LI, K, HT, HE, HN, PB, out, ovf); break;
                case 2: k_sweep<1, 4, 1><<<blocks, G>>>(il, L, LI, K, HT, HE, HN, PB, out, ovf); break;
                case 3: k_sweep<1, 8, 0><<<blocks, G>>>(il, L, LI, K, HT, HE, HN, PB, out, ovf); break;
                default: k_sweep<1, 2, 1><<<blocks, G>>>(il, L, LI, K, HT, HE, HN, PB, out, ovf); break;
            }
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            uint32_t o = 0;
            CK(hipMemcpy(&o, ovf, 4, hipMemcpyDeviceToHost));
            std::vector<uint32_t> hn(waves);
            CK(hipMemcpy(hn.data(), HN, (size_t)waves * 4, hipMemcpyDeviceToHost));
            double avg = 0.0;
            for (uint32_t i = 0; i < waves; ++i) avg += hn[i];
            unsigned long long cs = 0ull;
            std::vector<unsigned long long> ho(L);
            CK(hipMemcpy(ho.data(), out, (size_t)L * 8, hipMemcpyDeviceToHost));
            for (uint32_t i = 0; i < L; ++i) cs += ho[i];
            printf("{\"variant\": \"%s\", \"lanes\": %u, \"launch\": %u, \"ms\": %.4f, \"pool_end_avg_items\": %.1f, \"overflow_items\": %u, \"checksum\": %llu}\n",
                   vname[v], L, l, ms, avg / waves, o, cs);
            fflush(stdout);
        }
    }
    return 0;
}

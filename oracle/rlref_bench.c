/*
 * rlref_bench.c — CPU baseline timer (test/bench infrastructure only): "ref_dense".
 *
 * Times the oracle's faithful single-env restatement of the reference training
 * loop (src/agent.rs:66-118 with src/agent/one_step_agent.rs:53-86; dense-array
 * Q, no per-step history Vecs) on host cores: `threads` independent env+agent
 * pairs, one per thread, no sharing — the reference itself is single-threaded
 * (SURVEY §5).  The eval interleave (src/agent.rs:107-113) runs when eval_at > 0
 * (the bins pass n/10).  Each thread trains `repeats` fresh agents of
 * n_episodes each.  The reference's own data structures (FxHashMap Q etc.)
 * are timed by ref_faithful.c ("ref_faithful").
 *
 * usage: rlref_bench <env> <map8x8> <slippery> <agent> <policy> <selector> <algo>
 *                    <n_episodes> <eval_at> <threads> [repeats] [planning_steps]
 * policy 2 (NeuralPolicy) takes src/bin/frozen_lake_neural.rs's network and decay:
 * DenseLayer(1, 32) -> leaky_relu6 -> DenseLayer(32, 4) -> linear on the scalar
 * observation, ε <- ε * exploration_time (0.5); planning_steps > 0 wraps the agent
 * in InternalModelAgent + RandomModel (src/bin/cliffwalking_model.rs:151-157).
 * prints one JSON line: {"steps":..,"seconds":..,"threads":..,"steps_per_sec":..}
 */
#include "rlref.h"
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

typedef struct {
    rlo_config c;
    uint64_t n_episodes, eval_at, steps, repeats;
    uint32_t planning;
    double seconds;
} job;

static void *run(void *p) {
    job *j = (job *)p;
    for (uint64_t k = 0; k < j->repeats; ++k) {
        double sec = 0.0;
        if (j->planning) {
            rlo_faithful *f = rlo_faithful_create(&j->c);
            rlo_faithful_set_planning(f, j->planning);
            struct timespec t0, t1;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            j->steps += rlo_faithful_train(f, j->n_episodes, j->eval_at);
            clock_gettime(CLOCK_MONOTONIC, &t1);
            sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
            rlo_faithful_destroy(f);
        } else {
            j->steps += rlo_faithful_bench(&j->c, j->n_episodes, j->eval_at, &sec);
        }
        j->seconds += sec;
    }
    return NULL;
}

int main(int argc, char **argv) {
    if (argc < 11) {
        fprintf(stderr, "usage: %s env map8x8 slippery agent policy selector algo n_episodes eval_at threads\n",
                argv[0]);
        return 2;
    }
    rlo_config c = {0};
    c.env = atoi(argv[1]); c.map8x8 = atoi(argv[2]); c.slippery = atoi(argv[3]);
    c.agent = atoi(argv[4]); c.policy = atoi(argv[5]); c.selector = atoi(argv[6]); c.algo = atoi(argv[7]);
    uint64_t n = strtoull(argv[8], NULL, 10), eval_at = strtoull(argv[9], NULL, 10);
    int threads = atoi(argv[10]);
    if (threads < 1) threads = 1;
    const uint64_t repeats = argc > 11 ? strtoull(argv[11], NULL, 10) : 1;
    /* CLI defaults of the reference bins: src/bin/frozen_lake.rs:35-73,84 */
    c.max_steps = 100; c.lr = 0.05; c.gamma = 0.95; c.lambda_ = 0.5; c.eps0 = 1.0;
    c.eps_decay = 1.0 / (0.5 * (double)n); c.eps_final = 0.0; c.ucb_c = 0.5; c.q_default = 0.0;
    c.seed = 0x5EED; c.n_lanes = 1; c.group_size = 1; c.sync_every = 1; c.eval_episodes = 100;
    if (c.policy == RLO_POLICY_NEURAL) {   /* src/bin/frozen_lake_neural.rs:81,130-134,178-183 */
        c.net_input = RLO_INPUT_SCALAR; c.net_hidden = 32;
        c.net_act1 = RLO_ACT_LEAKY_RELU6; c.net_act2 = RLO_ACT_LINEAR;
        c.decay_kind = RLO_DECAY_MUL; c.eps_decay = 0.5;
    }
    const uint32_t planning = argc > 12 ? (uint32_t)strtoul(argv[12], NULL, 10) : 0u;
    job *jobs = (job *)calloc((size_t)threads, sizeof(job));
    pthread_t *tid = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < threads; ++i) {
        jobs[i].c = c;
        jobs[i].c.lane_offset = (uint64_t)i;
        jobs[i].n_episodes = n;
        jobs[i].eval_at = eval_at;
        jobs[i].repeats = repeats;
        jobs[i].planning = planning;
        pthread_create(&tid[i], NULL, run, &jobs[i]);
    }
    uint64_t steps = 0;
    for (int i = 0; i < threads; ++i) {
        pthread_join(tid[i], NULL);
        steps += jobs[i].steps;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    printf("{\"steps\": %llu, \"seconds\": %.6f, \"threads\": %d, \"steps_per_sec\": %.3f}\n",
           (unsigned long long)steps, sec, threads, (double)steps / sec);
    free(jobs); free(tid);
    return 0;
}

/*
 * san_driver.c — TEST INFRASTRUCTURE ONLY: runs the CPU oracle (rlref.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "race detection /
 * sanitizers").  Every fixture in tests/golden comes from
 * rlref.c's hand-managed buffers, so each code path a fixture uses is exercised
 * here: the faithful single-env loop (train / evaluate / reset, records, Dyna
 * planning, NeuralPolicy) and the batched schedule in private and shared mode,
 * both Q representations, the split merge (launch_groups / fold / apply_delta)
 * and the reset-and-step option — on every env, agent, policy, selector and
 * algorithm family.  Built by `make san` (oracle/Makefile) with
 * -fsanitize=address,undefined -fno-sanitize-recover=all, so the first error
 * aborts with a nonzero status; tests/test_oracle_sanitize.py runs it.
 *
 * usage: rlref_san [quick]   prints one line per family and "san ok" at the end
 */
#include "rlref.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static rlo_config cfg(int env, int map8, int slip, int agent, int policy, int sel, int algo, uint32_t lanes,
                      uint32_t g, uint32_t k) {
    rlo_config c;
    memset(&c, 0, sizeof c);
    c.env = env; c.map8x8 = map8; c.slippery = slip; c.max_steps = 100;
    c.agent = agent; c.policy = policy; c.selector = sel; c.algo = algo; c.decay_kind = RLO_DECAY_LINEAR;
    c.lr = 0.05; c.gamma = 0.95; c.lambda_ = 0.5; c.eps0 = 1.0; c.eps_decay = 1.0 / (0.5 * 40.0);
    c.eps_final = 0.0; c.ucb_c = 0.5; c.q_default = 0.0; c.seed = 0x5EED; c.lane_offset = 3;
    c.n_lanes = lanes; c.group_size = g; c.sync_every = k; c.eval_episodes = 5;
    c.net_input = (env == RLO_ENV_FROZEN_LAKE_EDITED || (env == RLO_ENV_FROZEN_LAKE && agent == 1)) ? RLO_INPUT_FL_OBS
                                                                                           : RLO_INPUT_SCALAR;
    c.net_hidden = 8; c.net_act1 = RLO_ACT_LEAKY_RELU6; c.net_act2 = RLO_ACT_LINEAR;
    return c;
}

static void faithful(const rlo_config *c, uint32_t plan) {
    rlo_faithful *f = rlo_faithful_create(c);
    if (!f) { fprintf(stderr, "faithful create failed: env %d agent %d policy %d sel %d algo %d\n", c->env, c->agent, c->policy, c->selector, c->algo); exit(3); }
    rlo_faithful_set_record(f, 1);
    if (plan) rlo_faithful_set_planning(f, plan);
    rlo_faithful_train(f, 40, 10);
    uint32_t S, A;
    rlo_env_dims(c, &S, &A);
    const uint64_t ne = rlo_faithful_n_episodes(f), ns = rlo_faithful_n_steps(f);
    double *rh = malloc(sizeof(double) * (ne + 1)), *te = malloc(sizeof(double) * (ns + 1));
    uint64_t *el = malloc(sizeof(uint64_t) * (ne + 1));
    rlo_faithful_histories(f, rh, el, te);
    const uint64_t nr = rlo_faithful_get_records(f, NULL, 0);
    rlo_record *rec = malloc(sizeof(rlo_record) * (nr + 1));
    rlo_faithful_get_records(f, rec, nr);
    rlo_faithful_evaluate(f, 10);
    double *q = malloc(sizeof(double) * 2 * S * A);
    rlo_faithful_get_q(f, q);
    rlo_faithful_reset(f);
    rlo_faithful_train(f, 5, 2);
    free(rh); free(te); free(el); free(rec); free(q);
    rlo_faithful_destroy(f);
}

static void batch(const rlo_config *c, int qmode, int reset_step, uint32_t plan) {
    rlo_batch *b = rlo_batch_create(c);
    if (!b) { fprintf(stderr, "batch create failed\n"); exit(3); }
    rlo_batch_set_record(b, 1);
    if (qmode) rlo_batch_set_q_mode(b, qmode);
    if (reset_step) rlo_batch_set_reset_step(b, 1);
    if (plan) (void)rlo_batch_set_planning(b, plan);
    rlo_batch_run(b, 2);
    rlo_batch_train_episodes(b, 6, 3);
    rlo_batch_evaluate(b, 2);
    uint32_t S, A;
    rlo_env_dims(c, &S, &A);
    const uint32_t P = c->policy == RLO_POLICY_DOUBLE ? 2 : 1;
    const uint64_t nr = rlo_batch_n_records(b);
    rlo_record *rec = malloc(sizeof(rlo_record) * (nr + 1));
    rlo_batch_take_records(b, rec, nr);
    const size_t nq = (size_t)P * S * A * (c->group_size == 1 ? c->n_lanes : 1);
    double *q = malloc(sizeof(double) * nq);
    rlo_batch_get_q(b, q);
    if (c->group_size > 1) {
        int64_t *raw = malloc(sizeof(int64_t) * P * S * A);
        rlo_batch_get_q_raw(b, raw);
        free(raw);
        uint8_t *fl = malloc((size_t)P * S * A);
        rlo_batch_get_qflags(b, fl);
        free(fl);
        /* the split merge a rank runs: groups -> [MAX] -> fold -> [SUM] -> apply */
        const uint64_t nw = rlo_batch_delta_words(b);
        int64_t *delta = calloc(nw, sizeof(int64_t));
        rlo_batch_launch_groups(b, delta);
        rlo_batch_fold(b, delta);
        rlo_batch_apply_delta(b, delta);
        free(delta);
        rlo_batch_set_merge_groups(b, 4096);
        rlo_batch_run(b, 1);
    }
    uint64_t *n = malloc(sizeof(uint64_t) * S * A * c->n_lanes), *t = malloc(sizeof(uint64_t) * c->n_lanes);
    rlo_batch_get_ucb(b, n, t);
    rlo_batch_set_ucb(b, n, t);
    double *eps = malloc(sizeof(double) * c->n_lanes);
    rlo_batch_lane_eps(b, eps);
    uint64_t st[16];
    rlo_batch_stats(b, st);
    rlo_batch_set_q(b, q);
    rlo_batch_set_selector(b, c->selector ^ 1);
    rlo_batch_set_algo(b, (c->algo + 1) % 3);
    rlo_batch_run(b, 1);
    rlo_batch_reset(b);
    rlo_batch_run(b, 1);
    free(rec); free(q); free(n); free(t); free(eps);
    rlo_batch_destroy(b);
}

int main(int argc, char **argv) {
    const int quick = argc > 1 && strcmp(argv[1], "quick") == 0;
    int families = 0;
    for (int env = 0; env <= RLO_ENV_FROZEN_LAKE_EDITED; ++env)
        for (int agent = 0; agent <= 1; ++agent)
            for (int policy = 0; policy <= 2; ++policy)
                for (int sel = 0; sel <= 1; ++sel)
                    for (int algo = 0; algo <= 2; ++algo) {
                        if (quick && (algo != 1 || sel != 0) && !(env == RLO_ENV_TAXI && sel == 1 && algo == 2))
                            continue;
                        const int map8 = env == RLO_ENV_FROZEN_LAKE || env == RLO_ENV_FROZEN_LAKE_EDITED;
                        const int slip = (env == RLO_ENV_FROZEN_LAKE && agent == 1) ? 1 : 0;
                        rlo_config c = cfg(env, map8, slip, agent, policy, sel, algo, 24, 1, 16);
                        faithful(&c, 0);
                        batch(&c, 0, 0, 0);
                        if (policy == RLO_POLICY_NEURAL) {   /* private agents only */
                            ++families;
                            continue;
                        }
                        if (agent == 0 && policy == 0 && sel == 0) {   /* Dyna (private) */
                            faithful(&c, 3);
                            batch(&c, 0, 0, 3);
                        }
                        rlo_config s = cfg(env, map8, slip, agent, policy, sel, algo, 150, 64, 8);
                        batch(&s, 0, 0, 0);            /* fixed point where proven, else f64 */
                        batch(&s, RLO_QMODE_F64, 0, 0);
                        if (sel == 0) batch(&s, 0, 1, 0);   /* reset-and-step */
                        ++families;
                    }
    printf("san ok: %d families\n", families);
    return 0;
}

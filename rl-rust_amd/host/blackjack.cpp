// blackjack — CLI mirror of src/bin/blackjack.rs, including the win-rate loop
// (:179-207): 1,000,000 episodes of get_action + env.step after each training
// run, classified by the final reward.  That loop is Agent::evaluate with
// per-episode outcomes, run on the device (lanes share the 1e6 episodes).
#include "cli_common.hpp"

int main(int argc, char **argv) {
    cli::Flags f("RLRust - BlackJack");
    cli::common_flags(f, false);
    f.parse(argc, argv);
    rl_env_config env{};
    env.kind = RL_ENV_BLACKJACK;
    return cli::guarded([&] {
        return cli::run_sweep(f, env, [&](rlamd::Agent &agent, const std::string &legend) {
            constexpr uint64_t LOOP_LEN = 1000000;
            const uint32_t L = agent.config().n_lanes;
            const uint64_t per_lane = (LOOP_LEN + L - 1) / L;
            agent.evaluate(per_lane);
            uint64_t wins = 0, losses = 0, draws = 0;
            for (const auto &e : agent.last_episodes()) {
                if (e.mode != RL_MODE_EVAL) continue;
                if (e.reward == 1.0) ++wins;
                else if (e.reward == -1.0) ++losses;
                else ++draws;
            }
            const double n = (double)(per_lane * L);
            std::printf("%s has win-rate of %s%%, loss-rate of %s%% and draw-rate %s%%\n", legend.c_str(),
                        cli::rust_f64((double)wins / n).c_str(), cli::rust_f64((double)losses / n).c_str(),
                        cli::rust_f64((double)draws / n).c_str());
            std::fflush(stdout);
        });
    });
}

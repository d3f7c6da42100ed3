// cliffwalking_model — CLI mirror of src/bin/cliffwalking_model.rs: one-step
// Q-learning vs the same agent inside InternalModelAgent + RandomModel with 10
// planning steps (Dyna-Q, :151-157), both ε-greedy.
#include "cli_common.hpp"

int main(int argc, char **argv) {
    cli::Flags f("RLRust - CliffWalking - model");
    cli::common_flags(f, true);
    f.parse(argc, argv);
    rl_env_config env{};
    env.kind = RL_ENV_CLIFF_WALKING;
    env.max_steps = (uint32_t)f.u64("max_steps");
    const std::vector<cli::AgentSpec> specs = {
        {RL_AGENT_ONE_STEP, 0, {{"ε-Greedy One-Step Qlearning", RL_SEL_EPS_GREEDY, RL_ALGO_QLEARNING}}},
        {RL_AGENT_ONE_STEP, 10, {{"ε-Greedy One-Step Dyna-Qlearning", RL_SEL_EPS_GREEDY, RL_ALGO_QLEARNING}}},
    };
    return cli::guarded([&] { return cli::run_agents(f, env, specs); });
}

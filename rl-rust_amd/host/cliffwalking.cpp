// cliffwalking — CLI mirror of src/bin/cliffwalking.rs (CliffWalkingEnv::new(max_steps))
#include "cli_common.hpp"

int main(int argc, char **argv) {
    cli::Flags f("RLRust - CliffWalking");
    cli::common_flags(f, true);
    f.parse(argc, argv);
    rl_env_config env{};
    env.kind = RL_ENV_CLIFF_WALKING;
    env.max_steps = (uint32_t)f.u64("max_steps");
    return cli::guarded([&] { return cli::run_sweep(f, env); });
}

// frozen_lake — CLI mirror of src/bin/frozen_lake.rs (flags :20-74, sweep :171-216)
#include "cli_common.hpp"

int main(int argc, char **argv) {
    cli::Flags f("RLRust - FrozenLake");
    f.flag("stochastic_env", "Should the env be stochastic");
    f.opt("map", "4x4", "Change the env's map, if possible");
    cli::common_flags(f, true);
    f.parse(argc, argv);
    rl_env_config env{};
    env.kind = RL_ENV_FROZEN_LAKE;
    env.map8x8 = f.str("map") == "4x4" ? 0 : 1;       // frozen_lake.rs:88-93: anything else is 8x8
    env.slippery = f.on("stochastic_env") ? 1 : 0;
    env.max_steps = (uint32_t)f.u64("max_steps");
    return cli::guarded([&] { return cli::run_sweep(f, env); });
}

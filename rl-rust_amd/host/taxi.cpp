// taxi — CLI mirror of src/bin/taxi.rs (TaxiEnv::new(max_steps), COUNT 6)
#include "cli_common.hpp"

int main(int argc, char **argv) {
    cli::Flags f("RLRust - Taxi");
    cli::common_flags(f, true);
    f.parse(argc, argv);
    rl_env_config env{};
    env.kind = RL_ENV_TAXI;
    env.max_steps = (uint32_t)f.u64("max_steps");
    return cli::guarded([&] { return cli::run_sweep(f, env); });
}

// rl_train_cliff_walking.hip — kernel instantiations for RL_ENV_CLIFF_WALKING (one translation unit per env
// so the 48 specialisations of each env compile in parallel).
#include "rl_train_impl.h"

namespace rlamd {
train_launch_fn train_table_cliff_walking(int agent, int policy, int sel, int algo, int priv) {
    return train_table_entry<RL_ENV_CLIFF_WALKING>(agent, policy, sel, algo, priv);
}
}  // namespace rlamd

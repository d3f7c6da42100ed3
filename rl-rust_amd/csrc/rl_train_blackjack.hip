// rl_train_blackjack.hip — kernel instantiations for RL_ENV_BLACKJACK (one translation unit per env
// so the 16 specialisations of each env compile in parallel).
#include "rl_train_impl.h"

namespace rlamd {
train_launch_fn train_table_blackjack(int agent, int policy, int sel, int priv) {
    return train_table_entry<RL_ENV_BLACKJACK>(agent, policy, sel, priv);
}
}  // namespace rlamd

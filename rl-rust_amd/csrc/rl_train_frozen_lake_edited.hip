// rl_train_frozen_lake_edited.hip — kernel instantiations for RL_ENV_FROZEN_LAKE_EDITED
// (src/env/frozen_lake_edited.rs; one translation unit per env, compiled in parallel).
#include "rl_train_impl.h"

namespace rlamd {
train_launch_fn train_table_frozen_lake_edited(int agent, int policy, int sel, int algo, int priv) {
    return train_table_entry<RL_ENV_FROZEN_LAKE_EDITED>(agent, policy, sel, algo, priv);
}
}  // namespace rlamd

// Instance group E of the register-chained PPO kernel (see ppo_rc_instances.h).
#include "ppo_rc_kernel.h"
#include "ppo_rc_instances.h"

namespace ia {
namespace rc {
IA_RC_GROUP_E(IA_RC_INSTANTIATE)
}  // namespace rc
}  // namespace ia

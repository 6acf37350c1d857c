// Dev probe (not product): compile the Fp2 leaves in a minimal translation unit and read their
// register counts from the assembly (tools/micro/leaf_regs.sh).
#include "lsg_kcommon.hpp"
__global__ void LSG_KERNEL_ATTR k_leaf_probe(int n, uint32_t* m) {
  LANE_ITEM(n);
  (void)lead;
  const fp2_t a = lane_load<fp2_t>(m, 2 * item), b = lane_load<fp2_t>(m, 2 * item + 1);
  lane_store(m, 2 * item, fp2_add(fp2_mul(a, b), fp2_sqr(a)));
}

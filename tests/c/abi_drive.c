/* A plain C client of the drop-in boundary (include/lmm/lmm_system.h + lmm_hip.h): it builds the
 * reference's maxmin_test.cpp:17-42 system (C = 3, penalties 1 and 2 -> values 2 and 1) and the
 * exec-ptask L07 system of examples/s4u/exec-ptask/s4u-exec-ptask.tesh:9-12 through the System ABI,
 * solves both on the device, reads the values, the opaque ids and the device saturated set, and exits 0
 * iff they match.  Compiled by tests/test_abi.py (CPU), run by tests/test_gpu_parity.py (MI355X). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include "lmm/lmm_hip.h"
#include "lmm/lmm_system.h"

static int check(int ok, const char* what) {
  if (!ok)
    fprintf(stderr, "FAIL: %s (%s)\n", what, lmm_last_error());
  return ok ? 0 : 1;
}

int main(void) {
  int bad = 0;
  static int action1, action2;
  if (lmm_config_set("maxmin/solver:hip") != 0)
    return 2;
  /* maxmin_test.cpp:17-42 */
  lmm_sys* s = lmm_system_new(0, 0);
  int64_t c = lmm_constraint_new(s, 3.0);
  int64_t r1 = lmm_variable_new_id(s, &action1, 1.0, -1.0, 1);
  int64_t r2 = lmm_variable_new_id(s, &action2, 2.0, -1.0, 1);
  bad |= check(lmm_expand(s, c, r1, 1.0) == 0 && lmm_expand(s, c, r2, 1.0) == 0, "expand");
  bad |= check(lmm_solve(s) == 0, "solve");
  bad |= check(fabs(lmm_variable_get_value(s, r1) - 2.0) < 1e-12, "rho1 == 2");
  bad |= check(fabs(lmm_variable_get_value(s, r2) - 1.0) < 1e-12, "rho2 == 1");
  bad |= check(lmm_variable_get_id(s, r1) == &action1 && lmm_variable_get_id(s, r2) == &action2, "ids");
  uint8_t sat = 0;
  bad |= check(lmmhip_get_saturated(lmm_system_device_ctx(s), &sat) == 0 && sat == 1, "saturated set");
  lmm_system_free(s);
  /* s4u-exec-ptask.tesh:9-12: 3 x 1 Gflop on 100 Mf hosts, 10 MB per pair on the 100 kBps bus */
  lmm_sys* f = lmm_system_new(0, 1);
  int64_t h[3], bus;
  for (int i = 0; i < 3; i++)
    h[i] = lmm_constraint_new(f, 100e6);
  bus = lmm_constraint_new(f, 100e3);
  int64_t v = lmm_variable_new(f, 1.0, -1.0, 4);
  for (int i = 0; i < 3; i++)
    bad |= check(lmm_expand(f, h[i], v, 1e9) == 0, "expand cpu");
  for (int k = 0; k < 3; k++)
    bad |= check(lmm_expand_add(f, bus, v, 1e7) == 0, "expand_add bus");
  bad |= check(lmm_solve(f) == 0, "fair solve");
  const double x = lmm_variable_get_value(f, v);
  bad |= check(fabs(x * 1e9 - 3333333.333333) < 5e-7 && fabs(x * 3e7 - 100000.0) < 5e-7, "speed_used / bus");
  lmm_system_free(f);
  printf(bad ? "abi_drive: FAILED\n" : "abi_drive: ok\n");
  return bad;
}

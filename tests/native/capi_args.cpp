// TEST INFRASTRUCTURE ONLY -- the C ABI's argument validation (include/hmpc.h)
// under AddressSanitizer + UndefinedBehaviorSanitizer on the host (built by
// tests/test_sanitizers.py with hipcc, -fsanitize= after -Xarch_host).  No GPU
// is needed: every call below must be rejected (or report "no device")
// before any kernel launch, and nothing may touch memory it does not own.
#include <stdio.h>
#include <stdint.h>

#include "../../include/hmpc.h"

static int fails = 0;
#define EXPECT(cond)                                          \
  do {                                                        \
    if (!(cond)) {                                            \
      fprintf(stderr, "FAILED: %s (line %d)\n", #cond, __LINE__); \
      ++fails;                                                \
    }                                                         \
  } while (0)

int main() {
  const double Jinv[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, rh[3] = {0, 0, 0};
  hmpc_ctx* c = nullptr;
  EXPECT(hmpc_version() >= 10000);
  int Ns[8];
  EXPECT(hmpc_supported_horizons(3, Ns, 8) >= 1);
  EXPECT(hmpc_supported_horizons(7, Ns, 8) == 0);
  EXPECT(hmpc_supported_horizons(3, nullptr, 0) >= 1);
  // hmpc_create: every invalid argument is HMPC_ERR_ARG / _UNSUPPORTED
  EXPECT(hmpc_create(nullptr, 3, 10, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 0, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 3, 10, 0.02, 7.5, 9.807, 1.0, nullptr, rh, 0, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 3, 10, 0.02, 7.5, 9.807, 1.0, Jinv, nullptr, 0, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 5, 10, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 0, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 4, 12, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 0, 0) == HMPC_ERR_UNSUPPORTED);   // CasADi variant: N <= 11
  EXPECT(hmpc_create(&c, 3, 0, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 0, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 3, 10, 0.0, 7.5, 9.807, 1.0, Jinv, rh, 0, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 3, 10, 0.02, -1.0, 9.807, 1.0, Jinv, rh, 0, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 3, 10, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 9, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_create(&c, 3, 1000, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 0, 0) == HMPC_ERR_UNSUPPORTED);
  EXPECT(c == nullptr);
  // no GPU in this container: a valid create reports HMPC_ERR_HIP and no context
  const int rc = hmpc_create(&c, 3, 10, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 0, 0);
  EXPECT(rc == HMPC_OK || rc == HMPC_ERR_HIP);
  // NULL contexts everywhere
  double d[16] = {0};
  int32_t s[4] = {0};
  double ms = 0;
  EXPECT(hmpc_destroy(nullptr) == HMPC_ERR_ARG);
  EXPECT(hmpc_solve_batch(nullptr, 1, d, d, d, d, d, nullptr, d, d, d, s, s, nullptr) == HMPC_ERR_ARG);
  EXPECT(hmpc_solve_batch_host(nullptr, 1, d, d, d, d, d, nullptr, d, d, d, s, s) == HMPC_ERR_ARG);
  EXPECT(hmpc_mpcontrol_batch(nullptr, 1, 1, d, d, d, d, nullptr, d, d, d, s, s, nullptr) == HMPC_ERR_ARG);
  EXPECT(hmpc_mpcontrol_plan_batch(nullptr, 1, 1, d, d, d, 10, 0, 0, 1, d, 0, nullptr, d, d, d, s, s,
                                   nullptr) == HMPC_ERR_ARG);
  EXPECT(hmpc_plant_batch(nullptr, 1, 1, 1e-3, d, d, d, 6, d, 0, 0, nullptr, nullptr, nullptr) == HMPC_ERR_ARG);
  EXPECT(hmpc_convert_batch(nullptr, 1, d, d, nullptr) == HMPC_ERR_ARG);
  EXPECT(hmpc_set_precision(nullptr, 0) == HMPC_ERR_ARG);
  EXPECT(hmpc_time_solve_batch(nullptr, 1, d, d, d, d, d, nullptr, d, d, d, s, s, 1, nullptr, &ms) ==
         HMPC_ERR_ARG);
  EXPECT(hmpc_last_error(nullptr)[0] == '\0');
  EXPECT(hmpc_kernel_name(nullptr)[0] == '\0');
  int64_t ot = -1;
  EXPECT(hmpc_overflow_total(nullptr, &ot) == HMPC_ERR_ARG);
  if (rc == HMPC_OK && c) {   // (a GPU host) the argument checks of a live context
    EXPECT(hmpc_solve_batch(c, -1, d, d, d, d, d, nullptr, d, d, d, s, s, nullptr) == HMPC_ERR_ARG);
    EXPECT(hmpc_solve_batch(c, 1, nullptr, d, d, d, d, nullptr, d, d, d, s, s, nullptr) == HMPC_ERR_ARG);
    EXPECT(hmpc_set_precision(c, 99) == HMPC_ERR_ARG);
    EXPECT(hmpc_overflow_total(c, nullptr) == HMPC_ERR_ARG);
    EXPECT(hmpc_overflow_total(c, &ot) == HMPC_OK && ot == 0);
    EXPECT(hmpc_time_solve_batch(c, 1, d, d, d, d, d, nullptr, d, d, d, s, s, 0, nullptr, &ms) == HMPC_ERR_ARG);
    EXPECT(hmpc_destroy(c) == HMPC_OK);
  }
  printf("capi_args: %d failure(s)\n", fails);
  return fails ? 1 : 0;
}

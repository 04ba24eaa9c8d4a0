/*
 * TEST INFRASTRUCTURE ONLY -- memory-safety self-test of the oracle's C port
 * (oracle/hmpc_port.c) under AddressSanitizer + UndefinedBehaviorSanitizer
 * (oracle/Makefile target `sanitize`, run by tests/test_sanitizers.py).
 *
 * Drives hport_solve_batch over synthetic hopping windows at several horizons
 * (N = 1, 2, 10, 20, 60), both variants, stance / swing / mixed contact
 * schedules, an infeasible start (z < 0.1) and B = 0, with OpenMP threads.
 * Parity is tested elsewhere (tests/test_oracle_port.py); here only that every
 * access stays in bounds and no arithmetic is undefined.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

long hport_solve_batch(int variant, int N, double t, double m, double g, double mu_default,
                       const double* Jinv, const double* rh, int uref_aliased, long B,
                       const double* x_in, const double* x_lin, const double* x_ref,
                       const double* pf, const double* C, const double* mu, double* u, double* x,
                       double* obj, int* status, int* iters, int nthreads);

static int run(int variant, int N, long B, int infeasible) {
  const double Jinv[9] = {13.13, -0.02, -0.36, -0.02, 21.99, 0.03, -0.36, 0.03, 13.11};
  const double rh[3] = {-2.663114e-5, -4.435752e-5, -6.61082088e-3};
  double* x_in = calloc((size_t)(B ? B : 1) * 12, sizeof(double));
  double* x_lin = calloc((size_t)(B ? B : 1) * 12 * (N + 1), sizeof(double));
  double* x_ref = calloc((size_t)(B ? B : 1) * 12 * N, sizeof(double));
  double* pf = calloc((size_t)(B ? B : 1) * 3 * N, sizeof(double));
  double* C = calloc((size_t)(B ? B : 1) * N, sizeof(double));
  double* mu = calloc((size_t)(B ? B : 1), sizeof(double));
  double* u = calloc((size_t)(B ? B : 1) * 6 * N, sizeof(double));
  double* x = calloc((size_t)(B ? B : 1) * 12 * (N + 1), sizeof(double));
  double* obj = calloc((size_t)(B ? B : 1), sizeof(double));
  int* st = calloc((size_t)(B ? B : 1), sizeof(int));
  int* it = calloc((size_t)(B ? B : 1), sizeof(int));
  for (long b = 0; b < B; ++b) {
    const double ph = 0.37 * (double)b;
    x_in[12 * b + 0] = 0.01 * sin(ph);
    x_in[12 * b + 2] = infeasible && b == 0 ? 0.05 : 0.27 + 0.05 * sin(2.0 * ph);
    x_in[12 * b + 5] = 0.1 * cos(ph);
    x_in[12 * b + 8] = -0.3 * cos(ph);
    x_in[12 * b + 9] = 0.5 * sin(3.0 * ph);
    memcpy(x_lin + 12 * (N + 1) * b, x_in + 12 * b, 12 * sizeof(double));
    for (int k = 0; k < N; ++k) {
      double* r = x_ref + 12 * N * b + 12 * k;
      r[0] = 0.005 * k;
      r[2] = 0.27 + 0.1 * sin(0.3 * k);
      r[5] = 0.01 * k;
      memcpy(x_lin + 12 * (N + 1) * b + 12 * (k + 1), r, 12 * sizeof(double));
      pf[3 * N * b + 3 * k] = 0.005 * k;
      C[N * b + k] = ((k + b) / 3) % 2 ? 1.0 : 0.0;   /* mixed stance / swing */
    }
    if (b % 3 == 0) for (int k = 0; k < N; ++k) C[N * b + k] = 1.0;   /* all stance */
    mu[b] = 0.3 + 0.1 * (double)(b % 9);
  }
  const long solved = hport_solve_batch(variant, N, 0.02, 7.5, 9.807, 1.0, Jinv, rh, 1, B, x_in, x_lin,
                                        x_ref, pf, C, mu, u, x, obj, st, it, 4);
  for (long b = 0; b < B; ++b)
    if (st[b] == 0 && !isfinite(obj[b])) { fprintf(stderr, "non-finite objective\n"); return 1; }
  printf("variant %d N %d B %ld: %ld solved\n", variant, N, B, solved);
  free(x_in); free(x_lin); free(x_ref); free(pf); free(C); free(mu); free(u); free(x); free(obj);
  free(st); free(it);
  return 0;
}

int main(void) {
  int rc = 0;
  const int Ns[] = {1, 2, 10, 20, 60};
  for (int v = 2; v <= 3; ++v)
    for (int i = 0; i < 5; ++i) rc |= run(v, Ns[i], Ns[i] == 60 ? 6 : 24, i == 2);
  rc |= run(3, 10, 0, 0);
  return rc;
}

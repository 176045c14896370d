/*
 * kf_dense_ref.c -- dense float64 textbook Kalman filter, batched over robots.
 * TEST INFRASTRUCTURE ONLY: the long-horizon accuracy reference of tests/test_oracle_kf_long.py.
 * Nothing in the product links or calls it.
 *
 * The KF math has no reference counterpart; the north star defines it:
 *     predict:  x <- F x (EKF: x <- f(x)),   P <- F P F^T + Q
 *     update:   S = H P H^T + R,  K = P H^T S^-1,  x += K y,  P -= K H P
 * This file evaluates exactly those formulas with full n x n matrices: S^-1 through an LU
 * factorisation with partial pivoting (K^T = S^-1 (H P)), the P update in Joseph form
 * (I - K H) P (I - K H)^T + K R K^T.  It shares no code and no operation order with the fp32
 * restatement (oracle/fmskf_oracle.c: LDL^T / sequential scalar updates, packed P) and
 * restates oracle/kf_ref.py (numpy) in C so that 60 000 ticks x 1000+ robots run in seconds;
 * tests/test_oracle_kf_long.py checks the two restatements against each other.
 *
 * State layout: x [N][n] and full P [N][n][n] row-major per robot; z [m][N] planes (float64).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define NMAX 12
#define MMAX 8

static const double kPi = 3.141592653589793;

static double wrap_innov(double a) {
  if (a > kPi) return a - 2.0 * kPi;
  if (a < -kPi) return a + 2.0 * kPi;
  return a;
}
static double wrap_state(double a) {
  if (a >= kPi) return a - 2.0 * kPi;
  if (a < -kPi) return a + 2.0 * kPi;
  return a;
}

/* C = A B, A [r][k], B [k][c] (row strides = column counts) */
static void mm(int r, int k, int c, const double *A, const double *B, double *C) {
  for (int i = 0; i < r; i++)
    for (int j = 0; j < c; j++) {
      double s = 0.0;
      for (int t = 0; t < k; t++) s += A[i * k + t] * B[t * c + j];
      C[i * c + j] = s;
    }
}
/* C = A B^T, A [r][k], B [c][k] */
static void mmt(int r, int k, int c, const double *A, const double *B, double *C) {
  for (int i = 0; i < r; i++)
    for (int j = 0; j < c; j++) {
      double s = 0.0;
      for (int t = 0; t < k; t++) s += A[i * k + t] * B[j * k + t];
      C[i * c + j] = s;
    }
}

/* solve S X = B for X [m][c] (S [m][m] copied), LU with partial pivoting; 0 if singular */
static int lu_solve(int m, const double *S_in, int c, double *B) {
  double S[MMAX * MMAX];
  memcpy(S, S_in, sizeof(double) * m * m);
  for (int k = 0; k < m; k++) {
    int p = k;
    for (int i = k + 1; i < m; i++)
      if (fabs(S[i * m + k]) > fabs(S[p * m + k])) p = i;
    if (S[p * m + k] == 0.0) return 0;
    if (p != k) {
      for (int j = 0; j < m; j++) {
        double t = S[k * m + j];
        S[k * m + j] = S[p * m + j];
        S[p * m + j] = t;
      }
      for (int j = 0; j < c; j++) {
        double t = B[k * c + j];
        B[k * c + j] = B[p * c + j];
        B[p * c + j] = t;
      }
    }
    for (int i = k + 1; i < m; i++) {
      const double f = S[i * m + k] / S[k * m + k];
      for (int j = k; j < m; j++) S[i * m + j] -= f * S[k * m + j];
      for (int j = 0; j < c; j++) B[i * c + j] -= f * B[k * c + j];
    }
  }
  for (int k = m - 1; k >= 0; k--)
    for (int j = 0; j < c; j++) {
      double s = B[k * c + j];
      for (int t = k + 1; t < m; t++) s -= S[k * m + t] * B[t * c + j];
      B[k * c + j] = s / S[k * m + k];
    }
  return 1;
}

/* x, P (full) <- the Joseph-form update with H [m][n], R [m][m], innovation y [m] */
static void update(int n, int m, double *x, double *P, const double *H, const double *R, const double *y) {
  double HP[MMAX * NMAX], S[MMAX * MMAX], Kt[MMAX * NMAX], K[NMAX * MMAX];
  mm(m, n, n, H, P, HP);
  mmt(m, n, m, HP, H, S);
  for (int i = 0; i < m * m; i++) S[i] += R[i];
  memcpy(Kt, HP, sizeof(double) * m * n);  /* K^T = S^-1 H P  (S symmetric) */
  if (!lu_solve(m, S, n, Kt)) return;
  for (int i = 0; i < n; i++)
    for (int a = 0; a < m; a++) K[i * m + a] = Kt[a * n + i];
  for (int i = 0; i < n; i++) {
    double s = 0.0;
    for (int a = 0; a < m; a++) s += K[i * m + a] * y[a];
    x[i] += s;
  }
  double IKH[NMAX * NMAX], T1[NMAX * NMAX], T2[NMAX * NMAX], KR[NMAX * MMAX];
  mm(n, m, n, K, H, IKH);
  for (int i = 0; i < n * n; i++) IKH[i] = -IKH[i];
  for (int i = 0; i < n; i++) IKH[i * n + i] += 1.0;
  mm(n, n, n, IKH, P, T1);
  mmt(n, n, n, T1, IKH, T2);
  mm(n, m, m, K, R, KR);
  mmt(n, m, n, KR, K, T1);
  for (int i = 0; i < n * n; i++) P[i] = T2[i] + T1[i];
}

static void predict_cov(int n, double *P, const double *F, const double *Q) {
  double T1[NMAX * NMAX];
  mm(n, n, n, F, P, T1);
  mmt(n, n, n, T1, F, P);
  for (int i = 0; i < n * n; i++) P[i] += Q[i];
}

/* ---- KF6: x = (px, py, th, vx, vy, w); z = (th, w, vx_w, vy_w) ---------------------------- */
void dref_kf6_step(int64_t nr, double *x, double *P, const double *z, const uint8_t *valid,
                   const double *Q /*[36]*/, const double *R /*[16]*/, double dt) {
  double H[4 * 6] = {0}, F[36] = {0};
  const int hs[4] = {2, 5, 3, 4};
  for (int a = 0; a < 4; a++) H[a * 6 + hs[a]] = 1.0;
  for (int i = 0; i < 6; i++) F[i * 6 + i] = 1.0;
  for (int i = 0; i < 3; i++) F[i * 6 + i + 3] = dt;
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < nr; r++) {
    double *xr = x + r * 6, *Pr = P + r * 36;
    if (!valid || valid[r]) {
      double y[4];
      for (int a = 0; a < 4; a++) y[a] = z[a * nr + r] - xr[hs[a]];
      y[0] = wrap_innov(y[0]);
      update(6, 4, xr, Pr, H, R, y);
    }
    double xn[6];
    for (int i = 0; i < 6; i++) {
      double s = 0.0;
      for (int j = 0; j < 6; j++) s += F[i * 6 + j] * xr[j];
      xn[i] = s;
    }
    xn[2] = wrap_state(xn[2]);
    memcpy(xr, xn, sizeof(xn));
    predict_cov(6, Pr, F, Q);
  }
}

/* ---- EKF9: x = (px, py, th, vbx, vby, w, bw, abx, aby); z = (th, w + bw, abx, aby, vbx, vby) -- */
void dref_ekf9_step(int64_t nr, double *x, double *P, const double *z, const uint8_t *valid,
                    const double *Q /*[81]*/, const double *R /*[36]*/, double dt) {
  double H[6 * 9] = {0};
  H[0 * 9 + 2] = 1.0;
  H[1 * 9 + 5] = 1.0;
  H[1 * 9 + 6] = 1.0;
  H[2 * 9 + 7] = 1.0;
  H[3 * 9 + 8] = 1.0;
  H[4 * 9 + 3] = 1.0;
  H[5 * 9 + 4] = 1.0;
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < nr; r++) {
    double *xr = x + r * 9, *Pr = P + r * 81;
    if (!valid || valid[r]) {
      double y[6], hx[6];
      hx[0] = xr[2];
      hx[1] = xr[5] + xr[6];
      hx[2] = xr[7];
      hx[3] = xr[8];
      hx[4] = xr[3];
      hx[5] = xr[4];
      for (int a = 0; a < 6; a++) y[a] = z[a * nr + r] - hx[a];
      y[0] = wrap_innov(y[0]);
      update(9, 6, xr, Pr, H, R, y);
    }
    const double th = xr[2], vbx = xr[3], vby = xr[4];
    const double c = cos(th), s = sin(th);
    const double vwx = vbx * c - vby * s, vwy = vbx * s + vby * c;
    double F[81] = {0};
    for (int i = 0; i < 9; i++) F[i * 9 + i] = 1.0;
    F[0 * 9 + 2] = -vwy * dt;
    F[0 * 9 + 3] = c * dt;
    F[0 * 9 + 4] = -s * dt;
    F[1 * 9 + 2] = vwx * dt;
    F[1 * 9 + 3] = s * dt;
    F[1 * 9 + 4] = c * dt;
    F[2 * 9 + 5] = dt;
    F[3 * 9 + 7] = dt;
    F[4 * 9 + 8] = dt;
    xr[0] += vwx * dt;
    xr[1] += vwy * dt;
    xr[2] = wrap_state(xr[2] + xr[5] * dt);
    xr[3] += xr[7] * dt;
    xr[4] += xr[8] * dt;
    predict_cov(9, Pr, F, Q);
  }
}

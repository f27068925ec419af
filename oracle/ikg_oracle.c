/*
 * CPU ORACLE — test infrastructure only (tests/, smoke(), bench.py's
 * cpu_baseline leg).  Never linked into or called by libikgrasp.so.
 *
 * Plain-C fp64 restatement of the reference grasp-pose IK loop
 * (/root/reference/inverse_geometry.py:41-100, collision term excluded) with
 * the Pinocchio semantics it calls:
 *   framesForwardKinematics (:58)    -> fk(): oMi[j] = oMi[parent] * (placement_j * R_axis(q_j))
 *   log(oMhand^-1 * oMtarget) (:66)  -> log6() (Pinocchio log3/log6 branches)
 *   computeFrameJacobian LOCAL (:75) -> frame_jacobian(): backward pass,
 *                                       col_i = iMf.actInv(S_i), iMf <- liMi * iMf
 *   pinv(J) @ e (:83)                -> J^T (J J^T)^-1 e by a 12x12 Cholesky
 *                                       (equal to the pseudo-inverse for full-row-rank J)
 *   integrate + clip (:86, :89)      -> q + dq*DT, clipped to the URDF limits
 * The model tables are transcribed from NextageaOpen.urdf:580-730 and
 * cube_small.urdf:34-47 (same numbers as oracle/ik_oracle.py).
 * Parity: pinned to KAT-1/KAT-2 by tests/test_oracle_c.py.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NQ 15

static const int PARENT[NQ] = {-1, 0, 1, 0, 3, 4, 5, 6, 7, 0, 9, 10, 11, 12, 13};
static const int AXIS[NQ] = {2, 2, 1, 2, 1, 1, 0, 1, 2, 2, 1, 1, 0, 1, 2};
static const double ORIGIN[NQ][3] = {
    {0.0, 0.0, 0.267},      {0.0, 0.0, 0.302},     {0.0, 0.0, 0.08},   {0.04, 0.135, 0.1015},
    {0.0, 0.0, 0.066},      {0.0, 0.095, -0.25},   {0.1805, 0.0, -0.03}, {0.1495, 0.0, 0.0},
    {0.0, 0.0, -0.1335},    {0.04, -0.135, 0.1015}, {0.0, 0.0, 0.066},  {0.0, -0.095, -0.25},
    {0.1805, 0.0, -0.03},   {0.1495, 0.0, 0.0},    {0.0, 0.0, -0.1335}};
static const double LOWER[NQ] = {-3.14159, -1.22173, -0.401425, -1.5707963, -2.44346, -1.22173, -3.1415926, -3.57792,
                                 -2.7123889, -1.570796, -2.44346, -1.22173, -1.74532, -3.5779, -2.712388};
static const double UPPER[NQ] = {3.14159, 1.22173, 1.308997, 1.5707963, 1.0471975, 1.5707963, 1.7453292, 1.134464,
                                 2.7123889, 1.570796, 1.047197, 1.570796, 3.141592, 1.134464, 2.712388};
static const double ROBOT_Z = 0.85; /* config.py:33 */
static const int FRAME_JOINT[2] = {8, 14};
static const double FRAME_T[2][3] = {{0.082, 0.05, -0.02}, {0.082, -0.05, -0.02}};
static const double HOOK_T[2][3] = {{0.0, 0.05, 0.0}, {0.0, -0.05, 0.0}};

typedef struct {
  double R[3][3];
  double t[3];
} se3;

/* urdfdom rpy -> quaternion (normalised) -> Eigen matrix, yaw only */
static void rpy_yaw(double yaw, double R[3][3]) {
  double z = sin(yaw / 2.0), w = cos(yaw / 2.0);
  double n = sqrt(z * z + w * w);
  z /= n;
  w /= n;
  double tz = 2.0 * z;
  double twz = tz * w, tzz = tz * z;
  R[0][0] = 1.0 - tzz;
  R[0][1] = -twz;
  R[0][2] = 0.0;
  R[1][0] = twz;
  R[1][1] = 1.0 - tzz;
  R[1][2] = 0.0;
  R[2][0] = 0.0;
  R[2][1] = 0.0;
  R[2][2] = 1.0;
}

static void mul(const se3* a, const se3* b, se3* c) {
  se3 r;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) r.R[i][j] = a->R[i][0] * b->R[0][j] + a->R[i][1] * b->R[1][j] + a->R[i][2] * b->R[2][j];
    r.t[i] = a->t[i] + (a->R[i][0] * b->t[0] + a->R[i][1] * b->t[1] + a->R[i][2] * b->t[2]);
  }
  *c = r;
}

static void inv(const se3* a, se3* c) {
  se3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.R[i][j] = a->R[j][i];
  for (int i = 0; i < 3; ++i) r.t[i] = -(r.R[i][0] * a->t[0] + r.R[i][1] * a->t[1] + r.R[i][2] * a->t[2]);
  *c = r;
}

/* liMi = placement_j * R_axis(q_j) */
static void joint_local(int j, double q, se3* out) {
  double s = sin(q), c = cos(q);
  memset(out, 0, sizeof(*out));
  int a = AXIS[j];
  int b = (a + 1) % 3, d = (a + 2) % 3;
  out->R[a][a] = 1.0;
  out->R[b][b] = c;
  out->R[b][d] = -s;
  out->R[d][b] = s;
  out->R[d][d] = c;
  for (int i = 0; i < 3; ++i) out->t[i] = ORIGIN[j][i];
  if (j == 0) out->t[2] = ROBOT_Z + ORIGIN[0][2];
}

static void fk(const double* q, se3* oMi) {
  for (int j = 0; j < NQ; ++j) {
    se3 l;
    joint_local(j, q[j], &l);
    if (PARENT[j] < 0)
      oMi[j] = l;
    else
      mul(&oMi[PARENT[j]], &l, &oMi[j]);
  }
}

static void frame_placement_local(int h, se3* f) {
  rpy_yaw(1.5708, f->R);
  for (int i = 0; i < 3; ++i) f->t[i] = FRAME_T[h][i];
}

static void log6(const se3* M, double e[6]) {
  const double pi = 3.14159265358979323846;
  const double (*R)[3] = M->R;
  double tr = R[0][0] + R[1][1] + R[2][2];
  double theta = tr > 3.0 ? 0.0 : (tr < -1.0 ? pi : acos((tr - 1.0) / 2.0));
  double w[3];
  if (theta >= pi - 1e-2) {
    double cphi = cos(theta - pi);
    double beta = theta * theta / (1.0 + cphi);
    double t0 = (R[0][0] + cphi) * beta, t1 = (R[1][1] + cphi) * beta, t2 = (R[2][2] + cphi) * beta;
    w[0] = (R[2][1] > R[1][2] ? 1.0 : -1.0) * (t0 > 0 ? sqrt(t0) : 0.0);
    w[1] = (R[0][2] > R[2][0] ? 1.0 : -1.0) * (t1 > 0 ? sqrt(t1) : 0.0);
    w[2] = (R[1][0] > R[0][1] ? 1.0 : -1.0) * (t2 > 0 ? sqrt(t2) : 0.0);
  } else {
    const double prec3 = 1.220703125e-04; /* eps^(1/4) */
    double t = (theta > prec3 ? theta / sin(theta) : 1.0) / 2.0;
    w[0] = t * (R[2][1] - R[1][2]);
    w[1] = t * (R[0][2] - R[2][0]);
    w[2] = t * (R[1][0] - R[0][1]);
  }
  double t2 = theta * theta, alpha, beta;
  if (theta < 1.220703125e-04) {
    alpha = 1.0 - t2 / 12.0 - t2 * t2 / 720.0;
    beta = 1.0 / 12.0 + t2 / 720.0;
  } else {
    double st = sin(theta), ct = cos(theta);
    alpha = theta * st / (2.0 * (1.0 - ct));
    beta = 1.0 / t2 - st / (2.0 * theta * (1.0 - ct));
  }
  const double* p = M->t;
  double wp = w[0] * p[0] + w[1] * p[1] + w[2] * p[2];
  double cx = w[1] * p[2] - w[2] * p[1], cy = w[2] * p[0] - w[0] * p[2], cz = w[0] * p[1] - w[1] * p[0];
  e[0] = alpha * p[0] - 0.5 * cx + beta * wp * w[0];
  e[1] = alpha * p[1] - 0.5 * cy + beta * wp * w[1];
  e[2] = alpha * p[2] - 0.5 * cz + beta * wp * w[2];
  e[3] = w[0];
  e[4] = w[1];
  e[5] = w[2];
}

/* LOCAL frame Jacobian of hand h into rows J[0..5][*] */
static void frame_jacobian(const double* q, int h, double J[6][NQ]) {
  se3 iMf;
  frame_placement_local(h, &iMf);
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < NQ; ++c) J[r][c] = 0.0;
  for (int i = FRAME_JOINT[h]; i >= 0; i = PARENT[i]) {
    int a = AXIS[i];
    /* actInv(S): lin = R^T (-(t x e_a)), ang = R^T e_a */
    double ea[3] = {0, 0, 0};
    ea[a] = 1.0;
    const double* t = iMf.t;
    double v[3] = {-(t[1] * ea[2] - t[2] * ea[1]), -(t[2] * ea[0] - t[0] * ea[2]), -(t[0] * ea[1] - t[1] * ea[0])};
    for (int r = 0; r < 3; ++r) {
      J[r][i] = iMf.R[0][r] * v[0] + iMf.R[1][r] * v[1] + iMf.R[2][r] * v[2];
      J[3 + r][i] = iMf.R[a][r];
    }
    se3 l;
    joint_local(i, q[i], &l);
    mul(&l, &iMf, &iMf);
  }
}

/* dq = J^T (J J^T)^-1 e, J 12xNQ; returns 0 if J J^T is not positive definite */
static int min_norm_step(double J[12][NQ], const double e[12], double dq[NQ]) {
  double A[12][12], y[12];
  for (int r = 0; r < 12; ++r)
    for (int c = 0; c <= r; ++c) {
      double s = 0.0;
      for (int k = 0; k < NQ; ++k) s += J[r][k] * J[c][k];
      A[r][c] = s;
    }
  for (int k = 0; k < 12; ++k) {
    double d = A[k][k];
    for (int j = 0; j < k; ++j) d -= A[k][j] * A[k][j];
    if (!(d > 0.0)) return 0;
    d = sqrt(d);
    A[k][k] = d;
    for (int i = k + 1; i < 12; ++i) {
      double v = A[i][k];
      for (int j = 0; j < k; ++j) v -= A[i][j] * A[k][j];
      A[i][k] = v / d;
    }
  }
  for (int i = 0; i < 12; ++i) {
    double v = e[i];
    for (int j = 0; j < i; ++j) v -= A[i][j] * y[j];
    y[i] = v / A[i][i];
  }
  for (int i = 11; i >= 0; --i) {
    double v = y[i];
    for (int j = i + 1; j < 12; ++j) v -= A[j][i] * y[j];
    y[i] = v / A[i][i];
  }
  for (int k = 0; k < NQ; ++k) {
    double s = 0.0;
    for (int r = 0; r < 12; ++r) s += J[r][k] * y[r];
    dq[k] = s;
  }
  return 1;
}

static void hand_errors(const double* q, const se3 tgt[2], double e[12], double n[2]) {
  se3 oMi[NQ];
  fk(q, oMi);
  for (int h = 0; h < 2; ++h) {
    se3 f, oMf, hinv, M;
    frame_placement_local(h, &f);
    mul(&oMi[FRAME_JOINT[h]], &f, &oMf);
    inv(&oMf, &hinv);
    mul(&hinv, &tgt[h], &M);
    log6(&M, e + 6 * h);
    double s = 0.0;
    for (int i = 0; i < 6; ++i) s += e[6 * h + i] * e[6 * h + i];
    n[h] = sqrt(s);
  }
}

static void solve_one(const double* target, const double* q0, int max_iters, double eps, double dt, double* q_out,
                      uint8_t* conv, int32_t* iters, double* err) {
  se3 cube, hook, tgt[2];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) cube.R[i][j] = target[3 * i + j];
  for (int i = 0; i < 3; ++i) cube.t[i] = target[9 + i];
  for (int h = 0; h < 2; ++h) {
    if (h == 0) {
      memset(&hook, 0, sizeof(hook));
      hook.R[0][0] = hook.R[1][1] = hook.R[2][2] = 1.0;
    } else {
      rpy_yaw(-3.14, hook.R);
    }
    for (int i = 0; i < 3; ++i) hook.t[i] = HOOK_T[h][i];
    mul(&cube, &hook, &tgt[h]);
  }
  double q[NQ], e[12], n[2];
  memcpy(q, q0, sizeof(q));
  int it = 0, ok = 0;
  for (;;) {
    hand_errors(q, tgt, e, n);
    if (it >= max_iters) break;
    if (n[0] < eps && n[1] < eps) {
      ok = 1;
      break;
    }
    double J[12][NQ], dq[NQ];
    frame_jacobian(q, 0, (double(*)[NQ])J[0]);
    frame_jacobian(q, 1, (double(*)[NQ])J[6]);
    if (!min_norm_step(J, e, dq)) break;
    for (int k = 0; k < NQ; ++k) {
      double v = q[k] + dq[k] * dt;
      v = v > LOWER[k] ? v : LOWER[k];
      q[k] = v < UPPER[k] ? v : UPPER[k];
    }
    ++it;
  }
  memcpy(q_out, q, sizeof(q));
  *conv = (uint8_t)ok;
  *iters = it;
  err[0] = n[0];
  err[1] = n[1];
}

/* Batched entry (one problem per thread, `nthreads` OpenMP threads). */
int ikg_oracle_solve(const double* targets, const double* q0, int64_t q0_stride, int64_t B, int max_iters,
                     double eps, double dt, double* q_out, uint8_t* conv, int32_t* iters, double* err,
                     int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t i = 0; i < B; ++i)
    solve_one(targets + 12 * i, q0 + q0_stride * i, max_iters, eps, dt, q_out + NQ * i, conv + i, iters + i,
              err + 2 * i);
  return 0;
}

int ikg_oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

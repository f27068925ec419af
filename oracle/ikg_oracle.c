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
 * With a collision scene (ikg_oracle_solve_collision) the stop test also
 * requires collision(q) to be false (:70), restating oracle/collision_oracle.py.
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

/* Evaluation options (test infrastructure, tests/test_c_oracle.py,
 * tests/test_gpu_fullbatch.py).  0 = the reference's own formulas.
 *   ORC_ACC_LOG6: log3/log6 evaluated without the cancellation of the
 *     reference's acos((tr-1)/2) and 1-cos(theta) (theta = atan2(|skew|/2,
 *     (tr-1)/2), alpha = theta(1+cos)/(2 sin)): the same mathematics,
 *     rounded to ~1 ulp.  Near convergence (theta ~1e-3) the reference's theta
 *     carries ~1e-13 absolute / 1e-10 relative rounding noise.
 *   ORC_QR_STEP: the min-norm step pinv(J) e by Householder QR of J^T (error
 *     ~eps cond(J), the class of np.linalg.pinv's SVD) instead of the normal
 *     equations (~eps cond(J)^2).
 *   ORC_JITTER: every entry of every FK rotation is moved by 0 or +-1 ulp
 *     (a hash of jitter_seed, problem, update, joint, entry): the reference's
 *     own rounding envelope (how far its output moves when its FK rounds
 *     differently, as any other implementation's does). */
enum { ORC_ACC_LOG6 = 1, ORC_QR_STEP = 2, ORC_JITTER = 4 };
typedef struct {
  int flags;
  uint64_t seed; /* jitter: hash key, mixed with problem and update */
} orc_opts;

static uint64_t mix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

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

static void fk(const double* q, se3* oMi, const orc_opts* o, uint64_t key) {
  for (int j = 0; j < NQ; ++j) {
    se3 l;
    joint_local(j, q[j], &l);
    if (PARENT[j] < 0)
      oMi[j] = l;
    else
      mul(&oMi[PARENT[j]], &l, &oMi[j]);
    if (o && (o->flags & ORC_JITTER)) {
      uint64_t h = mix64(key ^ mix64((uint64_t)j + 0x51ull));
      for (int k = 0; k < 9; ++k, h >>= 2) {
        const int b = (int)(h & 3u); /* 0, 3: keep; 1: up; 2: down */
        double* r = &oMi[j].R[k / 3][k % 3];
        if (b == 1) *r = nextafter(*r, 2.0);
        if (b == 2) *r = nextafter(*r, -2.0);
      }
    }
  }
}

static void frame_placement_local(int h, se3* f) {
  rpy_yaw(1.5708, f->R);
  for (int i = 0; i < 3; ++i) f->t[i] = FRAME_T[h][i];
}

static void log6_acc(const se3* M, double e[6]);

static void log6(const se3* M, double e[6], int acc) {
  if (acc) {
    log6_acc(M, e);
    return;
  }
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

/* ORC_ACC_LOG6: the same log3/log6, every quantity from the rotation's skew
 * part and trace without cancellation (the near-pi axis as the reference). */
static void log6_acc(const se3* M, double e[6]) {
  const double pi = 3.14159265358979323846;
  const double (*R)[3] = M->R;
  const double sk[3] = {R[2][1] - R[1][2], R[0][2] - R[2][0], R[1][0] - R[0][1]};
  const double s = 0.5 * sqrt(sk[0] * sk[0] + sk[1] * sk[1] + sk[2] * sk[2]); /* sin theta */
  const double c = 0.5 * (R[0][0] + R[1][1] + R[2][2] - 1.0);                 /* cos theta */
  const double theta = atan2(s, c);
  double w[3];
  if (theta >= pi - 1e-2) {
    double cphi = -c;
    double beta = theta * theta / (1.0 + cphi);
    double t0 = (R[0][0] + cphi) * beta, t1 = (R[1][1] + cphi) * beta, t2 = (R[2][2] + cphi) * beta;
    w[0] = (R[2][1] > R[1][2] ? 1.0 : -1.0) * (t0 > 0 ? sqrt(t0) : 0.0);
    w[1] = (R[0][2] > R[2][0] ? 1.0 : -1.0) * (t1 > 0 ? sqrt(t1) : 0.0);
    w[2] = (R[1][0] > R[0][1] ? 1.0 : -1.0) * (t2 > 0 ? sqrt(t2) : 0.0);
  } else {
    const double t = s > 0.0 ? theta / (2.0 * s) : 0.5;
    for (int i = 0; i < 3; ++i) w[i] = t * sk[i];
  }
  const double t2 = theta * theta;
  double alpha, beta;
  if (theta < 1e-2) { /* series: dropped terms < 1e-16 relative */
    alpha = 1.0 - t2 / 12.0 - t2 * t2 / 720.0 - t2 * t2 * t2 / 30240.0;
    beta = 1.0 / 12.0 + t2 / 720.0 + t2 * t2 / 30240.0 + t2 * t2 * t2 / 1209600.0;
  } else {
    alpha = theta < 0.5 * pi ? theta * (1.0 + c) / (2.0 * s) : theta * s / (2.0 * (1.0 - c));
    beta = (1.0 - alpha) / t2;
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

/* ORC_QR_STEP: x = pinv(J) e for full-row-rank J by Householder QR of
 * A = J^T (NQ x 12): A = Q [R; 0], J = R^T Q^T, x = Q [R^-T e; 0]. */
static int qr_step(double J[12][NQ], const double e[12], double dq[NQ]) {
  double A[NQ][12], vs[12][NQ], beta[12];
  for (int i = 0; i < NQ; ++i)
    for (int j = 0; j < 12; ++j) A[i][j] = J[j][i];
  for (int k = 0; k < 12; ++k) {
    double nrm = 0.0;
    for (int i = k; i < NQ; ++i) nrm += A[i][k] * A[i][k];
    nrm = sqrt(nrm);
    if (!(nrm > 0.0)) return 0;
    const double alpha = A[k][k] > 0 ? -nrm : nrm;
    double vn = 0.0;
    for (int i = 0; i < NQ; ++i) vs[k][i] = i < k ? 0.0 : A[i][k];
    vs[k][k] -= alpha;
    for (int i = k; i < NQ; ++i) vn += vs[k][i] * vs[k][i];
    beta[k] = vn > 0.0 ? 2.0 / vn : 0.0;
    for (int j = k; j < 12; ++j) {
      double d = 0.0;
      for (int i = k; i < NQ; ++i) d += vs[k][i] * A[i][j];
      d *= beta[k];
      for (int i = k; i < NQ; ++i) A[i][j] -= d * vs[k][i];
    }
  }
  /* R^T y = e (R = upper 12 x 12 of A) */
  double x[NQ];
  for (int i = 0; i < 12; ++i) {
    double v = e[i];
    for (int j = 0; j < i; ++j) v -= A[j][i] * x[j];
    x[i] = v / A[i][i];
  }
  for (int i = 12; i < NQ; ++i) x[i] = 0.0;
  /* x <- Q x = H_0 H_1 ... H_11 x */
  for (int k = 11; k >= 0; --k) {
    double d = 0.0;
    for (int i = k; i < NQ; ++i) d += vs[k][i] * x[i];
    d *= beta[k];
    for (int i = k; i < NQ; ++i) x[i] -= d * vs[k][i];
  }
  for (int i = 0; i < NQ; ++i) dq[i] = x[i];
  return 1;
}

static void hand_errors(const double* q, const se3 tgt[2], double e[12], double n[2], const orc_opts* o,
                        uint64_t key) {
  se3 oMi[NQ];
  fk(q, oMi, o, key);
  for (int h = 0; h < 2; ++h) {
    se3 f, oMf, hinv, M;
    frame_placement_local(h, &f);
    mul(&oMi[FRAME_JOINT[h]], &f, &oMf);
    inv(&oMf, &hinv);
    mul(&hinv, &tgt[h], &M);
    log6(&M, e + 6 * h, o && (o->flags & ORC_ACC_LOG6));
    double s = 0.0;
    for (int i = 0; i < 6; ++i) s += e[6 * h + i] * e[6 * h + i];
    n[h] = sqrt(s);
  }
}

/* ---------------------------------------------------------------- collision term
 * Restates oracle/collision_oracle.py (itself the hpp-fcl semantics the
 * reference's tools.collision relies on, tools.py:25-35): a pair collides when
 * the two convex shapes intersect.  Sphere/sphere and sphere/box exact,
 * box/box by the 15-axis separating-axis test, every pair with a cylinder by
 * boolean GJK on support functions.  The scene (geometries in their parent
 * joint frames, active pairs; the target geometry is placed at the cube
 * target) comes from the caller (tests/golden/collision_scene.json). */
enum { K_SPHERE = 0, K_BOX = 1, K_CYL = 2, K_MESHBOX = 3 };

typedef struct {
  int n_geoms, n_pairs;
  const int32_t* kind;
  const int32_t* joint;  /* q index of the parent joint, -1 = world */
  const double* R;       /* [g][9] placement in the parent joint frame (world if joint < 0) */
  const double* t;       /* [g][3] */
  const double* dims;    /* [g][3] */
  const uint8_t* target; /* placed at the solve's cube target */
  const int32_t* pairs;  /* [k][2] */
} col_scene;

typedef struct {
  int kind;
  double R[3][3], t[3], d[3];
} shape;

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void cross3(const double* a, const double* b, double* c) {
  double r0 = a[1] * b[2] - a[2] * b[1], r1 = a[2] * b[0] - a[0] * b[2], r2 = a[0] * b[1] - a[1] * b[0];
  c[0] = r0, c[1] = r1, c[2] = r2;
}

static void support(const shape* g, const double* d, double* out) {
  if (g->kind == K_SPHERE) {
    double n = sqrt(dot3(d, d));
    for (int i = 0; i < 3; ++i) out[i] = g->t[i] + (n > 0 ? g->d[0] * d[i] / n : 0.0);
    return;
  }
  double dl[3], loc[3];
  for (int i = 0; i < 3; ++i) dl[i] = g->R[0][i] * d[0] + g->R[1][i] * d[1] + g->R[2][i] * d[2];
  if (g->kind == K_BOX || g->kind == K_MESHBOX) {
    for (int i = 0; i < 3; ++i) loc[i] = (dl[i] >= 0 ? 1.0 : -1.0) * g->d[i];
  } else {
    double rad = hypot(dl[0], dl[1]);
    loc[0] = rad > 0 ? g->d[0] * dl[0] / rad : 0.0;
    loc[1] = rad > 0 ? g->d[0] * dl[1] / rad : 0.0;
    loc[2] = dl[2] >= 0 ? g->d[1] : -g->d[1];
  }
  for (int i = 0; i < 3; ++i) out[i] = g->t[i] + g->R[i][0] * loc[0] + g->R[i][1] * loc[1] + g->R[i][2] * loc[2];
}

static void mink(const shape* a, const shape* b, const double* d, double* out) {
  double pa[3], pb[3], nd[3] = {-d[0], -d[1], -d[2]};
  support(a, d, pa);
  support(b, nd, pb);
  for (int i = 0; i < 3; ++i) out[i] = pa[i] - pb[i];
}

/* the simplex step of collision_oracle._do_simplex: s[0..n-1] oldest first,
 * s[n-1] newest; returns 1 when the origin is enclosed */
static int do_simplex(double s[4][3], int* n, double* d) {
  double* a = s[*n - 1];
  double ao[3] = {-a[0], -a[1], -a[2]};
  if (*n == 2) {
    double ab[3], t[3];
    for (int i = 0; i < 3; ++i) ab[i] = s[0][i] - a[i];
    if (dot3(ab, ao) > 0) {
      cross3(ab, ao, t);
      if (sqrt(dot3(t, t)) > 1e-15) {
        cross3(t, ab, d);
      } else { /* _perp(ab) */
        double e[3] = {fabs(ab[0]) < 0.9 ? 1.0 : 0.0, fabs(ab[0]) < 0.9 ? 0.0 : 1.0, 0.0};
        cross3(ab, e, d);
      }
      return 0; /* simplex [b, a] unchanged */
    }
    memcpy(s[0], a, sizeof(s[0]));
    *n = 1;
    memcpy(d, ao, sizeof(ao));
    return 0;
  }
  if (*n == 3) {
    double c[3], b[3], ab[3], ac[3], abc[3], t[3];
    memcpy(c, s[0], sizeof(c));
    memcpy(b, s[1], sizeof(b));
    for (int i = 0; i < 3; ++i) ab[i] = b[i] - a[i], ac[i] = c[i] - a[i];
    cross3(ab, ac, abc);
    cross3(abc, ac, t);
    if (dot3(t, ao) > 0) {
      if (dot3(ac, ao) > 0) {
        double a_[3];
        memcpy(a_, a, sizeof(a_));
        memcpy(s[0], c, sizeof(c));
        memcpy(s[1], a_, sizeof(a_));
        *n = 2;
        cross3(ac, ao, t);
        cross3(t, ac, d);
        return 0;
      }
      double a_[3];
      memcpy(a_, a, sizeof(a_));
      memcpy(s[0], b, sizeof(b));
      memcpy(s[1], a_, sizeof(a_));
      *n = 2;
      return do_simplex(s, n, d);
    }
    cross3(ab, abc, t);
    if (dot3(t, ao) > 0) {
      double a_[3];
      memcpy(a_, a, sizeof(a_));
      memcpy(s[0], b, sizeof(b));
      memcpy(s[1], a_, sizeof(a_));
      *n = 2;
      return do_simplex(s, n, d);
    }
    if (dot3(abc, ao) > 0) { /* [c, b, a] */
      memcpy(d, abc, sizeof(abc));
      return 0;
    }
    /* [b, c, a] */
    memcpy(s[0], b, sizeof(b));
    memcpy(s[1], c, sizeof(c));
    for (int i = 0; i < 3; ++i) d[i] = -abc[i];
    return 0;
  }
  double dd[3], c[3], b[3], ab[3], ac[3], ad[3], abc[3], acd[3], adb[3];
  memcpy(dd, s[0], sizeof(dd));
  memcpy(c, s[1], sizeof(c));
  memcpy(b, s[2], sizeof(b));
  for (int i = 0; i < 3; ++i) ab[i] = b[i] - a[i], ac[i] = c[i] - a[i], ad[i] = dd[i] - a[i];
  cross3(ab, ac, abc);
  cross3(ac, ad, acd);
  cross3(ad, ab, adb);
  double a_[3];
  memcpy(a_, a, sizeof(a_));
  if (dot3(abc, ao) > 0) {
    memcpy(s[0], c, sizeof(c)), memcpy(s[1], b, sizeof(b)), memcpy(s[2], a_, sizeof(a_));
    *n = 3;
    return do_simplex(s, n, d);
  }
  if (dot3(acd, ao) > 0) {
    memcpy(s[0], dd, sizeof(dd)), memcpy(s[1], c, sizeof(c)), memcpy(s[2], a_, sizeof(a_));
    *n = 3;
    return do_simplex(s, n, d);
  }
  if (dot3(adb, ao) > 0) {
    memcpy(s[0], b, sizeof(b)), memcpy(s[1], dd, sizeof(dd)), memcpy(s[2], a_, sizeof(a_));
    *n = 3;
    return do_simplex(s, n, d);
  }
  return 1;
}

static int gjk_intersect(const shape* a, const shape* b) {
  double s[4][3], d[3];
  for (int i = 0; i < 3; ++i) d[i] = a->t[i] - b->t[i];
  if (!(dot3(d, d) > 0)) d[0] = 1.0, d[1] = d[2] = 0.0;
  mink(a, b, d, s[0]);
  int n = 1;
  for (int i = 0; i < 3; ++i) d[i] = -s[0][i];
  for (int it = 0; it < 64; ++it) {
    if (dot3(d, d) < 1e-30) return 1;
    double p[3];
    mink(a, b, d, p);
    if (dot3(p, d) < 0) return 0;
    memcpy(s[n++], p, sizeof(p));
    if (do_simplex(s, &n, d)) return 1;
  }
  return 1;
}

static int box_box(const shape* a, const shape* b) {
  double ax[15][3];
  int k = 0;
  for (int i = 0; i < 3; ++i, ++k)
    for (int r = 0; r < 3; ++r) ax[k][r] = a->R[r][i];
  for (int i = 0; i < 3; ++i, ++k)
    for (int r = 0; r < 3; ++r) ax[k][r] = b->R[r][i];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j, ++k) {
      double ci[3] = {a->R[0][i], a->R[1][i], a->R[2][i]}, cj[3] = {b->R[0][j], b->R[1][j], b->R[2][j]};
      cross3(ci, cj, ax[k]);
    }
  double d[3] = {b->t[0] - a->t[0], b->t[1] - a->t[1], b->t[2] - a->t[2]};
  for (k = 0; k < 15; ++k) {
    double n = sqrt(dot3(ax[k], ax[k]));
    if (n < 1e-12) continue;
    double u[3] = {ax[k][0] / n, ax[k][1] / n, ax[k][2] / n};
    double r1 = 0, r2 = 0;
    for (int i = 0; i < 3; ++i) {
      double ci[3] = {a->R[0][i], a->R[1][i], a->R[2][i]}, cj[3] = {b->R[0][i], b->R[1][i], b->R[2][i]};
      r1 += a->d[i] * fabs(dot3(ci, u));
      r2 += b->d[i] * fabs(dot3(cj, u));
    }
    if (fabs(dot3(d, u)) > r1 + r2) return 0;
  }
  return 1;
}

static int collide(const shape* a, const shape* b) {
  int ka = a->kind, kb = b->kind;
  int bxa = ka == K_BOX || ka == K_MESHBOX, bxb = kb == K_BOX || kb == K_MESHBOX;
  if (ka == K_SPHERE && kb == K_SPHERE) {
    double d[3] = {a->t[0] - b->t[0], a->t[1] - b->t[1], a->t[2] - b->t[2]};
    return sqrt(dot3(d, d)) < a->d[0] + b->d[0];
  }
  if ((ka == K_SPHERE && bxb) || (kb == K_SPHERE && bxa)) {
    const shape* sp = ka == K_SPHERE ? a : b;
    const shape* bx = ka == K_SPHERE ? b : a;
    double w[3] = {sp->t[0] - bx->t[0], sp->t[1] - bx->t[1], sp->t[2] - bx->t[2]}, p[3], e2 = 0;
    for (int i = 0; i < 3; ++i) p[i] = bx->R[0][i] * w[0] + bx->R[1][i] * w[1] + bx->R[2][i] * w[2];
    for (int i = 0; i < 3; ++i) {
      double c = p[i] < -bx->d[i] ? -bx->d[i] : (p[i] > bx->d[i] ? bx->d[i] : p[i]);
      e2 += (p[i] - c) * (p[i] - c);
    }
    return sqrt(e2) < sp->d[0];
  }
  if (bxa && bxb) return box_box(a, b);
  return gjk_intersect(a, b);
}

/* tools.collision (tools.py:25-35) at q with the cube target `cube` */
static int collides(const col_scene* sc, const double* q, const se3* cube) {
  se3 oMi[NQ];
  fk(q, oMi, NULL, 0);
  shape g[64];
  if (sc->n_geoms > 64) return -1;
  for (int k = 0; k < sc->n_geoms; ++k) {
    se3 loc, w;
    for (int i = 0; i < 3; ++i) {
      for (int j = 0; j < 3; ++j) loc.R[i][j] = sc->R[9 * k + 3 * i + j];
      loc.t[i] = sc->t[3 * k + i];
    }
    if (sc->target[k])
      w = *cube;
    else if (sc->joint[k] < 0)
      w = loc;
    else
      mul(&oMi[sc->joint[k]], &loc, &w);
    g[k].kind = sc->kind[k];
    memcpy(g[k].R, w.R, sizeof(w.R));
    memcpy(g[k].t, w.t, sizeof(w.t));
    for (int i = 0; i < 3; ++i) g[k].d[i] = sc->dims[3 * k + i];
  }
  for (int p = 0; p < sc->n_pairs; ++p)
    if (collide(&g[sc->pairs[2 * p]], &g[sc->pairs[2 * p + 1]])) return 1;
  return 0;
}

static void solve_one(const double* target, const double* q0, int max_iters, double eps, double dt, double* q_out,
                      uint8_t* conv, int32_t* iters, double* err, const col_scene* sc, const orc_opts* o,
                      int64_t problem) {
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
    hand_errors(q, tgt, e, n, o, o ? mix64(o->seed ^ mix64((uint64_t)problem)) ^ (uint64_t)it : 0);
    if (it >= max_iters) break;
    /* :70 -- errors pass and (with a scene) not collision(q) */
    if (n[0] < eps && n[1] < eps && !(sc && collides(sc, q, &cube))) {
      ok = 1;
      break;
    }
    double J[12][NQ], dq[NQ];
    frame_jacobian(q, 0, J);
    frame_jacobian(q, 1, J + 6);
    if (!((o && (o->flags & ORC_QR_STEP)) ? qr_step(J, e, dq) : min_norm_step(J, e, dq))) break;
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
              err + 2 * i, NULL, NULL, i);
  return 0;
}

/* ikg_oracle_solve with evaluation options (orc_opts above); `first` is the
 * problem index of row 0 (the jitter hash key, so a subset reproduces a run). */
int ikg_oracle_solve_ex(const double* targets, const double* q0, int64_t q0_stride, int64_t B, int max_iters,
                        double eps, double dt, int flags, uint64_t seed, int64_t first, double* q_out, uint8_t* conv,
                        int32_t* iters, double* err, int nthreads) {
  const orc_opts o = {flags, seed};
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t i = 0; i < B; ++i)
    solve_one(targets + 12 * i, q0 + q0_stride * i, max_iters, eps, dt, q_out + NQ * i, conv + i, iters + i,
              err + 2 * i, NULL, &o, first + i);
  return 0;
}

/* The loop WITH the collision term (inverse_geometry.py:70, :97-98): the
 * scene arrays as col_scene documents them. */
int ikg_oracle_solve_collision(const double* targets, const double* q0, int64_t q0_stride, int64_t B, int max_iters,
                               double eps, double dt, int n_geoms, const int32_t* kind, const int32_t* joint,
                               const double* R, const double* t, const double* dims, const uint8_t* target,
                               int n_pairs, const int32_t* pairs, double* q_out, uint8_t* conv, int32_t* iters,
                               double* err, int nthreads) {
  if (n_geoms > 64) return -1;
  col_scene sc = {n_geoms, n_pairs, kind, joint, R, t, dims, target, pairs};
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
  for (int64_t i = 0; i < B; ++i)
    solve_one(targets + 12 * i, q0 + q0_stride * i, max_iters, eps, dt, q_out + NQ * i, conv + i, iters + i,
              err + 2 * i, &sc, NULL, i);
  return 0;
}

/* tools.collision alone, for the tests: out[i] = collision(q_i, target_i) */
int ikg_oracle_collision(const double* q, const double* targets, int64_t B, int n_geoms, const int32_t* kind,
                         const int32_t* joint, const double* R, const double* t, const double* dims,
                         const uint8_t* target, int n_pairs, const int32_t* pairs, uint8_t* out) {
  if (n_geoms > 64) return -1;
  col_scene sc = {n_geoms, n_pairs, kind, joint, R, t, dims, target, pairs};
  for (int64_t i = 0; i < B; ++i) {
    se3 cube;
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) cube.R[r][c] = targets[12 * i + 3 * r + c];
      cube.t[r] = targets[12 * i + 9 + r];
    }
    out[i] = (uint8_t)collides(&sc, q + NQ * i, &cube);
  }
  return 0;
}

int ikg_oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

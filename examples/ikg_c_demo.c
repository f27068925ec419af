/*
 * Minimal C caller of libikgrasp.so: the C-ABI with no
 * Python, no torch and no HIP headers.  Reads an ikg_model_desc (raw struct
 * bytes) and B cube targets (B x 12 doubles: R row-major, t), solves them from
 * q0 = 0 (the reference's robot.q0, inverse_geometry_TESTS.py / control.py:435)
 * with host pointers on device 0, and prints one line per target:
 *     <converged> <updates> <err_left> <err_right> <q_0> ... <q_{nq-1}>
 * Exit status 0 on success; 1 with ikg_last_error() on stderr otherwise.
 *
 *   ikg_c_demo desc.bin targets.bin [f64|f32] [specialize]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ikgrasp.h"

static void* slurp(const char* path, long* size) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  *size = ftell(f);
  fseek(f, 0, SEEK_SET);
  void* buf = malloc(*size > 0 ? (size_t)*size : 1);
  if (buf && fread(buf, 1, (size_t)*size, f) != (size_t)*size) {
    free(buf);
    buf = NULL;
  }
  fclose(f);
  return buf;
}

static int die(const char* what) {
  fprintf(stderr, "ikg_c_demo: %s: %s\n", what, ikg_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s desc.bin targets.bin [f64|f32] [specialize]\n", argv[0]);
    return 2;
  }
  const int f32 = argc > 3 && strcmp(argv[3], "f32") == 0;
  const int spec = argc > 4 && strcmp(argv[4], "specialize") == 0;
  long dsize = 0, tsize = 0;
  ikg_model_desc* desc = (ikg_model_desc*)slurp(argv[1], &dsize);
  double* targets = (double*)slurp(argv[2], &tsize);
  if (!desc || dsize != (long)sizeof(ikg_model_desc) || !targets || tsize % (12 * sizeof(double))) {
    fprintf(stderr, "ikg_c_demo: bad input files (desc %ld bytes, expected %zu)\n", dsize, sizeof(ikg_model_desc));
    return 2;
  }
  const int64_t B = tsize / (int64_t)(12 * sizeof(double));
  const int nq = desc->nq;
  ikg_model* model = NULL;
  if (ikg_model_create(desc, &model) != IKG_OK) return die("ikg_model_create");
  ikg_params p;
  ikg_params_default(&p); /* eps 1e-3, dt 1e-2, 1000 updates, lambda 0 */
  const int dtype = f32 ? IKG_F32 : IKG_F64;
  if (spec && ikg_model_specialize(model, 0, dtype, 0) != IKG_OK) return die("ikg_model_specialize");
  const size_t es = f32 ? sizeof(float) : sizeof(double);
  void* tg = targets;
  void* q0 = calloc((size_t)nq, es);
  void* q = malloc((size_t)(B * nq) * es);
  void* err = malloc((size_t)(B * 2) * es);
  uint8_t* conv = (uint8_t*)malloc((size_t)B);
  int32_t* iters = (int32_t*)malloc((size_t)B * sizeof(int32_t));
  if (f32) {
    float* t32 = (float*)malloc((size_t)(B * 12) * sizeof(float));
    for (int64_t i = 0; i < B * 12; ++i) t32[i] = (float)targets[i];
    tg = t32;
  }
  if (ikg_solve_batch(model, 0, dtype, tg, q0, 0, B, &p, q, conv, iters, err, NULL, IKG_FLAG_HOST_POINTERS) != IKG_OK)
    return die("ikg_solve_batch");
  for (int64_t b = 0; b < B; ++b) {
    const double e0 = f32 ? ((float*)err)[2 * b] : ((double*)err)[2 * b];
    const double e1 = f32 ? ((float*)err)[2 * b + 1] : ((double*)err)[2 * b + 1];
    printf("%d %d %.17g %.17g", conv[b], iters[b], e0, e1);
    for (int j = 0; j < nq; ++j) printf(" %.17g", f32 ? ((float*)q)[b * nq + j] : ((double*)q)[b * nq + j]);
    printf("\n");
  }
  ikg_model_destroy(model);
  return 0;
}

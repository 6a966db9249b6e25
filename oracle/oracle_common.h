/*
 * ORACLE -- test infrastructure only.  CPU restatement of the reference
 * algorithms used as the parity checker and as bench.py's cpu_baseline leg.
 * Never linked into, or called by, the product library.
 */
#ifndef ORACLE_COMMON_H_
#define ORACLE_COMMON_H_

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
  char name[128];
  int ndim;
  int64_t dims[4];
  int64_t numel;
  float* data;
} orc_tensor;

typedef struct {
  int count;
  orc_tensor* t;
} orc_weights;

/* RSPLWT01 blob reader (format: rspl-slam_amd/weights.py). Returns 0 on success. */
int orc_load_weights(const char* path, orc_weights* w);
void orc_free_weights(orc_weights* w);
const float* orc_get(const orc_weights* w, const char* name, int64_t expect_numel);

#endif

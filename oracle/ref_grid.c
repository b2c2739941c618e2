/*
 * ref_grid.c -- all-cores CPU baseline: the Go binding's multi-threaded MSM
 * (ref bindings/go/blst.go:2064-2197, breakdown :3181-3211, window size
 * :3213-3223) restated in C with pthreads, calling the REFERENCE's own
 * blst_p{1,2}s_tile_pippenger / _add_or_double / _double from libblst built
 * from /root/reference (oracle/Makefile).  TEST / BASELINE INFRASTRUCTURE ONLY:
 * loaded by bench.py's cpu_baseline leg and by tests, never by msm_blst_amd.
 *
 * The grid: nx point ranges x ny windows of `wnd` bits; a worker pool takes
 * tiles in order (top row first, as the Go code builds its grid) and the rows
 * are combined top-down with `wnd` doublings between rows, exactly the Go
 * collector's arithmetic (the result is the same point as
 * blst_p1s_mult_pippenger on the same inputs).
 *
 *   int ref_grid_msm(int group, void *ret, const void *points, size_t npoints,
 *                    const uint8_t *scalars, size_t nbits, int nthreads);
 * points: flat blst affine array; scalars: flat, stride (nbits+7)/8.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "blst.h"

static int bit_len(unsigned long v) {
  int n = 0;
  while (v) ++n, v >>= 1;
  return n;
}

static int go_window_size(size_t npoints) { /* blst.go:3213-3223 */
  int wbits = bit_len(npoints);
  if (wbits > 13) return wbits - 4;
  if (wbits > 5) return wbits - 3;
  return 2;
}

static void go_breakdown(int nbits, int window, int ncpus, int *nx_, int *ny_, int *wnd_) { /* blst.go:3181-3211 */
  int nx, ny, wnd;
  if (nbits > window * ncpus) {
    nx = 1;
    wnd = bit_len((unsigned)ncpus / 4);
    if (window + wnd > 18) {
      wnd = window - wnd;
    } else {
      wnd = (nbits / window + ncpus - 1) / ncpus;
      if ((nbits / (window + 1) + ncpus - 1) / ncpus < wnd) wnd = window + 1;
      else wnd = window;
    }
  } else {
    nx = 2;
    wnd = window - 2;
    while ((nbits / wnd + 1) * nx < ncpus) {
      nx += 1;
      wnd = window - bit_len(3 * (unsigned)nx / 2);
    }
    nx -= 1;
    wnd = window - bit_len(3 * (unsigned)nx / 2);
  }
  ny = nbits / wnd + 1;
  wnd = nbits / ny + 1;
  *nx_ = nx, *ny_ = ny, *wnd_ = wnd;
}

typedef struct {
  size_t x, dx, y;
  uint8_t point[288];
} tile_t;

typedef struct {
  int group;
  const uint8_t *points, *scalars;
  size_t nbytes, nbits, window;
  tile_t *grid;
  size_t total;
  size_t next;
  pthread_mutex_t mu;
} job_t;

static void *worker(void *arg) {
  job_t *J = (job_t *)arg;
  const size_t psz = 96 * (size_t)J->group;
  size_t scratch_bytes = J->group == 1 ? blst_p1s_mult_pippenger_scratch_sizeof(0)
                                       : blst_p2s_mult_pippenger_scratch_sizeof(0);
  limb_t *scratch = (limb_t *)malloc(scratch_bytes << (J->window - 1));
  for (;;) {
    pthread_mutex_lock(&J->mu);
    size_t k = J->next++;
    pthread_mutex_unlock(&J->mu);
    if (k >= J->total) break;
    tile_t *t = &J->grid[k];
    const void *pp[2] = {J->points + t->x * psz, NULL};
    const byte *sp[2] = {J->scalars + t->x * J->nbytes, NULL};
    if (J->group == 1)
      blst_p1s_tile_pippenger((blst_p1 *)t->point, (const blst_p1_affine *const *)pp, t->dx, sp, J->nbits, scratch,
                              t->y, J->window);
    else
      blst_p2s_tile_pippenger((blst_p2 *)t->point, (const blst_p2_affine *const *)pp, t->dx, sp, J->nbits, scratch,
                              t->y, J->window);
  }
  free(scratch);
  return NULL;
}

int ref_grid_msm(int group, void *ret, const void *points, size_t npoints, const uint8_t *scalars, size_t nbits,
                 int nthreads) {
  if ((group != 1 && group != 2) || npoints < 2 || nthreads < 1) return -1;
  int nx, ny, wnd;
  go_breakdown((int)nbits, go_window_size(npoints), nthreads, &nx, &ny, &wnd);
  job_t J;
  memset(&J, 0, sizeof J);
  J.group = group, J.points = (const uint8_t *)points, J.scalars = scalars;
  J.nbits = nbits, J.nbytes = (nbits + 7) / 8, J.window = (size_t)wnd;
  J.grid = (tile_t *)calloc((size_t)nx * ny, sizeof(tile_t));
  size_t dx = npoints / nx, y = (size_t)wnd * (ny - 1), total = 0;
  for (; total < (size_t)nx; ++total) J.grid[total].x = total * dx, J.grid[total].dx = dx, J.grid[total].y = y;
  J.grid[total - 1].dx = npoints - J.grid[total - 1].x;
  while (y > 0) {
    y -= wnd;
    for (int i = 0; i < nx; ++i, ++total)
      J.grid[total].x = J.grid[i].x, J.grid[total].dx = J.grid[i].dx, J.grid[total].y = y;
  }
  J.total = total;
  pthread_mutex_init(&J.mu, NULL);
  int nt = nthreads < (int)total ? nthreads : (int)total;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nt);
  for (int t = 0; t < nt; ++t) pthread_create(&th[t], NULL, worker, &J);
  for (int t = 0; t < nt; ++t) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&J.mu);
  /* rows top-down (blst.go:2173-2192): add the row's tiles, then wnd doublings */
  uint8_t acc[288];
  memset(acc, 0, sizeof acc);
  size_t row = 0;
  for (;;) {
    size_t yy = J.grid[row].y;
    for (; row < total && J.grid[row].y == yy; ++row) {
      if (group == 1) blst_p1_add_or_double((blst_p1 *)acc, (const blst_p1 *)acc, (const blst_p1 *)J.grid[row].point);
      else blst_p2_add_or_double((blst_p2 *)acc, (const blst_p2 *)acc, (const blst_p2 *)J.grid[row].point);
    }
    if (yy == 0) break;
    for (int j = 0; j < wnd; ++j) {
      if (group == 1) blst_p1_double((blst_p1 *)acc, (const blst_p1 *)acc);
      else blst_p2_double((blst_p2 *)acc, (const blst_p2 *)acc);
    }
  }
  memcpy(ret, acc, 144 * (size_t)group);
  free(J.grid);
  return 0;
}

int ref_grid_threads(size_t npoints, size_t nbits, int nthreads, int out[3]) {
  go_breakdown((int)nbits, go_window_size(npoints), nthreads, &out[0], &out[1], &out[2]);
  return 0;
}

/*
 * nlh_oracle.c -- CPU ORACLE (test infrastructure only; see nlh_oracle.h).
 *
 * Plain-C restatement of the reference serial solver
 *   /root/reference/src/2d_nonlocal_serial.cpp
 * with the per-term floating-point operation order kept exactly:
 *   sum_local       :256-270   res += ((J*c_2d)*(u_j - u_i))*(dh*dh), J = influence_function = 1.0
 *   sum_local_test  :235-252   res  = -(((2pi*sin(2pi*(t*dt)))*sin(2pi*(x*dh)))*sin(2pi*(y*dh)))
 *                              res -= ((1.0*c_2d)*(w~_j - w_i))*(dh*dh)
 *   w               :207-210   (cos(2pi*(t*dt))*sin(2pi*(x*dh)))*sin(2pi*(y*dh))
 *   boundary        :213-221   0 outside [0,nx)x[0,ny)
 *   len_1d_line     :231       (long)sqrt(eps*eps - dx*dx)
 *   do_work         :273-303   u' = u + sum_local*dt ; u' += sum_local_test*dt
 *   compute_l2/linf :96-113    sx-outer, sy-inner accumulation
 * Build with -ffp-contract=off (the reference is built without -march, so
 * x86-64 never contracts a*b+c into an FMA; CMakeLists.txt:23).
 *
 * sin(2pi*(x*dh)) is a pure function of x, so it is tabulated once per run;
 * the values are the same doubles the reference recomputes per neighbour.
 */
#define _GNU_SOURCE
#include "nlh_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

double nlh_oracle_c2d(const nlh_oracle_params *p) {
  if (p->influence == 1) return (p->k * 40) / pow(p->eps * p->dh, 4);
  return (p->k * 8) / pow(p->eps * p->dh, 4);
}

double nlh_oracle_influence(const nlh_oracle_params *p, long dx, long dy) {
  if (p->influence == 1) return 1.0 - sqrt((double)(dx * dx + dy * dy)) / (double)p->eps;
  return 1.0;
}

static long line_len(long eps, long dx) {
  return (long)sqrt((double)((eps * eps) - (dx * dx)));
}

long nlh_oracle_disk_count(long eps) {
  long n = 0;
  for (long dx = -eps; dx <= eps; ++dx) n += 2 * line_len(eps, labs(dx)) + 1;
  return n;
}

/* sin(2*pi*(i*dh)) for i in [lo, hi) -- the factor of w and of the IC */
static double *sin_table(long lo, long hi, double dh) {
  double *t = (double *)malloc(sizeof(double) * (size_t)(hi - lo));
  for (long i = lo; i < hi; ++i) t[i - lo] = sin(2 * M_PI * (i * dh));
  return t;
}

void nlh_oracle_test_init(const nlh_oracle_params *p, double *u) {
  for (long sx = 0; sx < p->nx; ++sx)
    for (long sy = 0; sy < p->ny; ++sy)
      u[sx + sy * p->nx] = sin(2 * M_PI * (sx * p->dh)) * sin(2 * M_PI * (sy * p->dh));
}

void nlh_oracle_exact(const nlh_oracle_params *p, long t, double *w) {
  const double ct = cos(2 * M_PI * (t * p->dt));
  for (long sx = 0; sx < p->nx; ++sx)
    for (long sy = 0; sy < p->ny; ++sy)
      w[sx + sy * p->nx] = ct * sin(2 * M_PI * (sx * p->dh)) * sin(2 * M_PI * (sy * p->dh));
}

/* ------------------------------------------------------------------------- */
typedef struct {
  const nlh_oracle_params *p;
  double c2d, dh2, st, ct;
  const double *sx_tab; /* index x + eps, covers [-eps, nx+eps) */
  const double *sy_tab; /* index y + eps, covers [-eps, ny+eps) */
} step_ctx;

/* sum_local (:256-270) */
static double sum_local(const step_ctx *c, const double *u, long x, long y) {
  const long nx = c->p->nx, ny = c->p->ny, eps = c->p->eps;
  const double ui = u[x + y * nx];
  double res = 0.0;
  for (long sx = x - eps; sx <= x + eps; ++sx) {
    const long len = line_len(eps, labs(x - sx));
    const int inx = (sx >= 0 && sx < nx);
    for (long sy = y - len; sy <= y + len; ++sy) {
      const double v = (inx && sy >= 0 && sy < ny) ? u[sx + sy * nx] : 0.0;
      res += ((nlh_oracle_influence(c->p, sx - x, sy - y) * c->c2d) * (v - ui)) * c->dh2;
    }
  }
  return res;
}

/* sum_local_test (:235-252), w via the tabulated sin factors */
static double sum_local_test(const step_ctx *c, long x, long y) {
  const long nx = c->p->nx, ny = c->p->ny, eps = c->p->eps;
  const double sxv = c->sx_tab[x + eps], syv = c->sy_tab[y + eps];
  double res = -(((2 * M_PI) * c->st) * sxv * syv);
  const double wpos = c->ct * sxv * syv;
  for (long sx = x - eps; sx <= x + eps; ++sx) {
    const long len = line_len(eps, labs(x - sx));
    const int inx = (sx >= 0 && sx < nx);
    for (long sy = y - len; sy <= y + len; ++sy) {
      const double wv =
          (inx && sy >= 0 && sy < ny) ? c->ct * c->sx_tab[sx + eps] * c->sy_tab[sy + eps] : 0.0;
      res -= ((nlh_oracle_influence(c->p, sx - x, sy - y) * c->c2d) * (wv - wpos)) * c->dh2;
    }
  }
  return res;
}

static void step_rect(const step_ctx *c, const double *u, double *un, long x0,
                      long x1, long y0, long y1) {
  const long nx = c->p->nx;
  const double dt = c->p->dt;
  for (long y = y0; y < y1; ++y)
    for (long x = x0; x < x1; ++x) {
      const long i = x + y * nx;
      un[i] = u[i] + (sum_local(c, u, x, y) * dt);
      if (c->p->test) un[i] += sum_local_test(c, x, y) * dt;
    }
}

static void ctx_init(step_ctx *c, const nlh_oracle_params *p) {
  c->p = p;
  c->c2d = nlh_oracle_c2d(p);
  c->dh2 = p->dh * p->dh;
  c->sx_tab = sin_table(-p->eps, p->nx + p->eps, p->dh);
  c->sy_tab = sin_table(-p->eps, p->ny + p->eps, p->dh);
}

static void ctx_time(step_ctx *c, long t) {
  c->st = sin(2 * M_PI * (t * c->p->dt));
  c->ct = cos(2 * M_PI * (t * c->p->dt));
}

static void ctx_free(step_ctx *c) {
  free((void *)c->sx_tab);
  free((void *)c->sy_tab);
}

/* ------------------------------------------------------------------------- */
/* persistent worker pool: tiles pulled from a shared counter, barrier/step   */
typedef struct {
  step_ctx *c;
  const double *u;
  double *un;
  long tiles_x, tiles_y, tw, th;
  long first, ntiles;  /* tiles first .. first+ntiles-1 of this step (all, or a timing sample) */
  long next_tile;
  pthread_mutex_t mu;
} tile_job;

static void *tile_worker(void *arg) {
  tile_job *j = (tile_job *)arg;
  const long ntiles = j->ntiles;
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const long k = j->next_tile++;
    pthread_mutex_unlock(&j->mu);
    if (k >= ntiles) break;
    const long t = j->first + k;
    const long gx = t % j->tiles_x, gy = t / j->tiles_x;
    const long x0 = gx * j->tw, y0 = gy * j->th;
    long x1 = x0 + j->tw, y1 = y0 + j->th;
    if (x1 > j->c->p->nx) x1 = j->c->p->nx;
    if (y1 > j->c->p->ny) y1 = j->c->p->ny;
    step_rect(j->c, j->u, j->un, x0, x1, y0, y1);
  }
  return NULL;
}

static void run_tiles_n(step_ctx *c, const double *u, double *un, long tiles_x,
                        long tiles_y, long first, long ntiles, int nthreads) {
  tile_job j;
  j.c = c;
  j.u = u;
  j.un = un;
  j.tiles_x = tiles_x;
  j.tiles_y = tiles_y;
  j.first = first;
  j.ntiles = ntiles;
  j.tw = (c->p->nx + tiles_x - 1) / tiles_x;
  j.th = (c->p->ny + tiles_y - 1) / tiles_y;
  j.next_tile = 0;
  pthread_mutex_init(&j.mu, NULL);
  if (nthreads <= 1) {
    tile_worker(&j);
  } else {
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int i = 0; i < nthreads; ++i) pthread_create(&th[i], NULL, tile_worker, &j);
    for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL); /* = barrier */
    free(th);
  }
  pthread_mutex_destroy(&j.mu);
}

static void run_tiles(step_ctx *c, const double *u, double *un, long tiles_x,
                      long tiles_y, int nthreads) {
  run_tiles_n(c, u, un, tiles_x, tiles_y, 0, tiles_x * tiles_y, nthreads);
}

void nlh_oracle_step(const nlh_oracle_params *p, long t, const double *u,
                     double *un, int nthreads) {
  step_ctx c;
  ctx_init(&c, p);
  ctx_time(&c, t);
  long rows = nthreads > 1 ? 4L * nthreads : 1;
  if (rows > p->ny) rows = p->ny > 0 ? p->ny : 1;
  run_tiles(&c, u, un, 1, rows, nthreads);
  ctx_free(&c);
}

void nlh_oracle_run(const nlh_oracle_params *p, long nt, double *u,
                    int nthreads) {
  const size_t n = (size_t)(p->nx * p->ny);
  double *b = (double *)malloc(sizeof(double) * (n ? n : 1));
  step_ctx c;
  ctx_init(&c, p);
  double *cur = u, *nxt = b;
  long rows = nthreads > 1 ? 4L * nthreads : 1;
  if (rows > p->ny) rows = p->ny > 0 ? p->ny : 1;
  for (long t = 0; t < nt; ++t) {
    ctx_time(&c, t);
    run_tiles(&c, cur, nxt, 1, rows, nthreads);
    double *tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  if (cur != u) memcpy(u, cur, sizeof(double) * n);
  ctx_free(&c);
  free(b);
}

void nlh_oracle_errors(const nlh_oracle_params *p, long time, const double *u,
                       double *l2, double *linf) {
  const double ct = cos(2 * M_PI * (time * p->dt));
  double e2 = 0, ei = 0;
  for (long sx = 0; sx < p->nx; ++sx) {
    const double sxv = sin(2 * M_PI * (sx * p->dh));
    for (long sy = 0; sy < p->ny; ++sy) {
      const double w = ct * sxv * sin(2 * M_PI * (sy * p->dh));
      const double d = u[sx + sy * p->nx] - w;
      e2 += d * d;
      const double a = fabs(d);
      ei = (a < ei) ? ei : a; /* std::max(abs(..), error_linf) */
    }
  }
  *l2 = e2;
  *linf = ei;
}

double nlh_oracle_run_tiled(const nlh_oracle_params *p, long nt, long tiles_x,
                            long tiles_y, double *u, int nthreads) {
  const size_t n = (size_t)(p->nx * p->ny);
  double *b = (double *)malloc(sizeof(double) * (n ? n : 1));
  step_ctx c;
  ctx_init(&c, p);
  double *cur = u, *nxt = b;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (long t = 0; t < nt; ++t) {
    ctx_time(&c, t);
    run_tiles(&c, cur, nxt, tiles_x, tiles_y, nthreads);
    double *tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (cur != u) memcpy(u, cur, sizeof(double) * n);
  ctx_free(&c);
  free(b);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* Timing sample of run_tiled's step t on a lattice too large to step whole
 * within the CPU baseline's budget: tiles first .. first+ntiles-1 (row-major)
 * of the same lattice, same tiling and threads; seconds.  The rest of the
 * next field is left uncomputed (it is only a timing). */
double nlh_oracle_time_tiles(const nlh_oracle_params *p, long t, long tiles_x, long tiles_y,
                             long first, long ntiles, const double *u, int nthreads) {
  const size_t n = (size_t)(p->nx * p->ny);
  double *b = (double *)calloc(n ? n : 1, sizeof(double));
  step_ctx c;
  ctx_init(&c, p);
  ctx_time(&c, t);
  if (first < 0) first = 0;
  if (first > tiles_x * tiles_y) first = tiles_x * tiles_y;
  if (ntiles > tiles_x * tiles_y - first) ntiles = tiles_x * tiles_y - first;
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  run_tiles_n(&c, u, b, tiles_x, tiles_y, first, ntiles, nthreads);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  ctx_free(&c);
  free(b);
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ------------------------------------------------------------------------- */
/* Compensated evaluation (test infrastructure): the same
 * explicit-Euler step as do_work (:273-303) -- the J = 1 disk sum of
 * sum_local (:256-270) and the manufactured source of sum_local_test
 * (:235-252) -- evaluated in x87 long double (64-bit significand) and rounded
 * to double ONCE per node and step:
 *   u' = u + dt ( c dh^2 (sum_disk u~_j - N u_i)
 *                 [ - (2 pi st) w0_i - c dh^2 (sum_disk w~_j - N w_i) ] )
 * The disk sum of a node is its 2E+1 row windows, row y+dy over columns
 * x - len(|dy|) .. x + len(|dy|) (the closed lattice disk is symmetric in x
 * and y, so this is the reference's set of points), each window a difference
 * of long-double prefix sums of the zero-extended row.  The result is the
 * reference's arithmetic without the rounding of its N(eps) sequential terms
 * (at eps >= 64 that rounding, not the GPU kernels', limits the comparison
 * with nlh_oracle_run): the target of the fast kernels' parity tests at the
 * stable dt.  J = 1 only (influence 0). */
typedef struct {
  const nlh_oracle_params *p;
  const double *u;
  double *un;
  const long double *pu;      /* row prefix sums of u, (nx + 1) per row */
  const long double *lw;      /* test mode: sum_disk W0~_j - N W0_i per node (W0 = sx sy), fixed */
  const long *len;            /* len(|d|), d = 0 .. eps */
  const double *sx_tab, *sy_tab;
  long double cdh2, st, ct;
  long y0, y1;
} comp_job;

static long double window_sum(const long double *prow, long nx, long x, long L) {
  long a = x - L, b = x + L + 1;
  if (a < 0) a = 0;
  if (b > nx) b = nx;
  return b > a ? prow[b] - prow[a] : 0.0L;
}

static void *comp_rows(void *arg) {
  const comp_job *j = (const comp_job *)arg;
  const long nx = j->p->nx, ny = j->p->ny, eps = j->p->eps;
  const long double N = (long double)nlh_oracle_disk_count(eps);
  const long double dt = (long double)j->p->dt;
  for (long y = j->y0; y < j->y1; ++y)
    for (long x = 0; x < nx; ++x) {
      long double su = 0.0L;
      for (long dy = -eps; dy <= eps; ++dy) {
        const long yy = y + dy;
        if (yy < 0 || yy >= ny) continue;
        su += window_sum(j->pu + yy * (nx + 1), nx, x, j->len[labs(dy)]);
      }
      const long double ui = (long double)j->u[x + y * nx];
      long double r = j->cdh2 * (su - N * ui);
      if (j->p->test) {
        /* w~ = ct W0~: its disk sum is ct times W0's, computed once */
        const long double w0 = (long double)j->sx_tab[x + eps] * (long double)j->sy_tab[y + eps];
        r += -(2.0L * (long double)M_PI * j->st) * w0 - j->cdh2 * (j->ct * j->lw[x + y * nx]);
      }
      j->un[x + y * nx] = (double)(ui + dt * r);
    }
  return NULL;
}

void nlh_oracle_run_compensated(const nlh_oracle_params *p, long nt, double *u, int nthreads) {
  const long nx = p->nx, ny = p->ny, eps = p->eps;
  const size_t n = (size_t)(nx * ny);
  double *b = (double *)malloc(sizeof(double) * (n ? n : 1));
  long double *pu = (long double *)malloc(sizeof(long double) * (size_t)(ny * (nx + 1)));
  long double *lw = p->test ? (long double *)malloc(sizeof(long double) * (n ? n : 1)) : NULL;
  long *len = (long *)malloc(sizeof(long) * (size_t)(eps + 1));
  for (long d = 0; d <= eps; ++d) len[d] = line_len(eps, d);
  step_ctx c;
  ctx_init(&c, p);
  if (lw) {
    /* sum_disk W0~_j - N W0_i once, from row windows of W0's prefix sums */
    const long double N = (long double)nlh_oracle_disk_count(eps);
    for (long y = 0; y < ny; ++y) {
      long double *r = pu + y * (nx + 1);
      r[0] = 0.0L;
      for (long x = 0; x < nx; ++x)
        r[x + 1] = r[x] + (long double)c.sx_tab[x + eps] * (long double)c.sy_tab[y + eps];
    }
    for (long y = 0; y < ny; ++y)
      for (long x = 0; x < nx; ++x) {
        long double sw = 0.0L;
        for (long dy = -eps; dy <= eps; ++dy) {
          const long yy = y + dy;
          if (yy >= 0 && yy < ny) sw += window_sum(pu + yy * (nx + 1), nx, x, len[labs(dy)]);
        }
        lw[x + y * nx] = sw - N * ((long double)c.sx_tab[x + eps] * (long double)c.sy_tab[y + eps]);
      }
  }
  if (nthreads < 1) nthreads = 1;
  if (nthreads > ny) nthreads = ny > 0 ? (int)ny : 1;
  pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
  comp_job *jobs = (comp_job *)malloc(sizeof(comp_job) * (size_t)nthreads);
  double *cur = u, *nxt = b;
  for (long t = 0; t < nt; ++t) {
    ctx_time(&c, t);
    for (long y = 0; y < ny; ++y) {
      long double *r = pu + y * (nx + 1);
      r[0] = 0.0L;
      for (long x = 0; x < nx; ++x) r[x + 1] = r[x] + (long double)cur[x + y * nx];
    }
    for (int i = 0; i < nthreads; ++i) {
      comp_job *j = &jobs[i];
      j->p = p;
      j->u = cur;
      j->un = nxt;
      j->pu = pu;
      j->lw = lw;
      j->len = len;
      j->sx_tab = c.sx_tab;
      j->sy_tab = c.sy_tab;
      j->cdh2 = (long double)c.c2d * (long double)c.dh2;
      j->st = (long double)c.st;
      j->ct = (long double)c.ct;
      j->y0 = ny * i / nthreads;
      j->y1 = ny * (i + 1) / nthreads;
      if (nthreads > 1)
        pthread_create(&th[i], NULL, comp_rows, j);
      else
        comp_rows(j);
    }
    if (nthreads > 1)
      for (int i = 0; i < nthreads; ++i) pthread_join(th[i], NULL);
    double *tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  if (cur != u) memcpy(u, cur, sizeof(double) * n);
  ctx_free(&c);
  free(jobs);
  free(th);
  free(len);
  free(lw);
  free(pu);
  free(b);
}

/* ------------------------------------------------------------------------- */
/* 1D solver (src/1d_nonlocal_serial.cpp)                                      */
double nlh_oracle_c1d(long eps, double k, double dx) {
  const long c = (long)((k * 3) / (pow(eps * dx, 3))); /* `long c_1d` (1d :57,74) */
  return (double)c;
}

void nlh_oracle_run_1d(long nx, long nt, long eps, double k, double dt, double dx, int test,
                       double *u) {
  const double c = nlh_oracle_c1d(eps, k, dx);
  double *s[2];
  s[0] = u;
  s[1] = (double *)malloc(sizeof(double) * (size_t)(nx > 0 ? nx : 1));
  double *sxt = sin_table(-eps, nx + eps, dx);
  for (long t = 0; t < nt; ++t) {
    const double *cur = s[t % 2];
    double *nxt = s[(t + 1) % 2];
    const double st = sin(2 * M_PI * (t * dt)), ct = cos(2 * M_PI * (t * dt));
    for (long x = 0; x < nx; ++x) {
      double res = 0.0;
      for (long sx = x - eps; sx <= x + eps; ++sx) {
        const double v = (sx >= 0 && sx < nx) ? cur[sx] : 0.0;
        res += ((1.0 * c) * (v - cur[x])) * dx;
      }
      nxt[x] = cur[x] + (res * dt);
      if (test) {
        double r2 = -(((2 * M_PI) * st) * sxt[x + eps]);
        const double wpos = ct * sxt[x + eps];
        for (long sx = x - eps; sx <= x + eps; ++sx) {
          const double wv = (sx >= 0 && sx < nx) ? ct * sxt[sx + eps] : 0.0;
          r2 -= ((1.0 * c) * (wv - wpos)) * dx;
        }
        nxt[x] += r2 * dt;
      }
    }
  }
  if (nt % 2) memcpy(u, s[1], sizeof(double) * (size_t)nx);
  free(s[1]);
  free(sxt);
}

void nlh_oracle_errors_1d(long nx, long time, double dt, double dx, const double *u,
                          double *l2, double *linf) {
  const double ct = cos(2 * M_PI * (time * dt));
  double e2 = 0, ei = 0;
  for (long sx = 0; sx < nx; ++sx) {
    const double w = ct * sin(2 * M_PI * (sx * dx));
    const double d = u[sx] - w;
    e2 += d * d;
    const double a = fabs(d);
    ei = (a < ei) ? ei : a;
  }
  *l2 = e2;
  *linf = ei;
}

/*
 * oracle_main.c — CLI around the CPU oracle (TEST INFRASTRUCTURE ONLY).
 * Prints one JSON object with the run's counts; used to generate and check
 * tests/golden fixtures (tools/make_golden.py).
 *
 *   kubeapi_oracle [-nc N] [-np N] [-ns N] [-nofail] [-notimeout]
 *                  [-nodeadlock] [-maxlevels L] [-maxdistinct D]
 *                  [-variant V] [-trace] [-threads T [-budget S]]
 */
#include "kubeapi_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int main(int argc, char **argv) {
  ko_config cfg = {1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 128, 0, 0, 0, 0};
  int print_trace = 0, threads = 0;
  double budget = 1e30;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "-nc") && i + 1 < argc) cfg.nc = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-np") && i + 1 < argc) cfg.np = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-ns") && i + 1 < argc) cfg.ns = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-nofail")) cfg.can_fail = 0;
    else if (!strcmp(argv[i], "-notimeout")) cfg.can_timeout = 0;
    else if (!strcmp(argv[i], "-nodeadlock")) cfg.check_deadlock = 0;
    else if (!strcmp(argv[i], "-notracestore")) cfg.keep_trace = 0;
    else if (!strcmp(argv[i], "-maxlevels") && i + 1 < argc) cfg.max_levels = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-maxdistinct") && i + 1 < argc) cfg.max_distinct = strtoull(argv[++i], 0, 10);
    else if (!strcmp(argv[i], "-variant") && i + 1 < argc) cfg.variant = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-lostupdate")) cfg.lost_update = 1;
    else if (!strcmp(argv[i], "-trace")) print_trace = 1;
    else if (!strcmp(argv[i], "-fp64")) cfg.fp_bits = 64;
    else if (!strcmp(argv[i], "-fp128")) cfg.fp_bits = 128;   /* (-threads: 128-bit keys) */
    else if (!strcmp(argv[i], "-fpsetlog2") && i + 1 < argc) cfg.fpset_log2 = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-progress")) cfg.progress = 1;
    else if (!strcmp(argv[i], "-threads") && i + 1 < argc) threads = atoi(argv[++i]);
    else if (!strcmp(argv[i], "-budget") && i + 1 < argc) budget = atof(argv[++i]);
    else { fprintf(stderr, "unknown arg %s\n", argv[i]); return 2; }
  }
  if (threads > 0) {          /* the multi-core comparator: counts and wall time only */
    ko_par_result p;
    double rate = ko_bench_parallel(&cfg, threads, budget, &p);
    printf("{\"nc\": %d, \"np\": %d, \"ns\": %d, \"threads\": %d, \"distinct\": %llu, "
           "\"generated\": %llu, \"levels\": %d, \"complete\": %d, \"set_full\": %d, "
           "\"seconds\": %.3f, \"distinct_per_s\": %.1f, \"fp_bits\": %d, \"depth\": %d, "
           "\"max_levels\": %d, \"level_width\": [",
           cfg.nc, cfg.np, cfg.ns, p.threads, (unsigned long long)p.distinct,
           (unsigned long long)p.generated, p.levels, p.complete, p.set_full, p.seconds, rate, p.fp_bits,
           p.depth, cfg.max_levels);
    for (int l = 0; l < p.depth; l++) printf("%s%llu", l ? ", " : "", (unsigned long long)p.level_width[l]);
    printf("]}\n");
    return 0;
  }
  static ko_result r;
  void *h = ko_run(&cfg, &r);
  printf("{\"nc\": %d, \"np\": %d, \"ns\": %d, \"can_fail\": %d, \"can_timeout\": %d,\n",
         cfg.nc, cfg.np, cfg.ns, cfg.can_fail, cfg.can_timeout);
  printf(" \"init\": %llu, \"generated\": %llu, \"distinct\": %llu, \"queue_left\": %llu,"
         " \"depth\": %d, \"complete\": %d, \"seconds\": %.3f,\n",
         (unsigned long long)r.init, (unsigned long long)r.generated,
         (unsigned long long)r.distinct, (unsigned long long)r.queue_left, r.depth, r.complete,
         r.seconds);
  printf(" \"act_gen\": {");
  for (int a = 0; a < KO_NACTIONS; a++)
    printf("%s\"%s\": %llu", a ? ", " : "", ko_action_name(a), (unsigned long long)r.act_gen[a]);
  printf("},\n \"act_dist\": {");
  for (int a = 0; a < KO_NACTIONS; a++)
    printf("%s\"%s\": %llu", a ? ", " : "", ko_action_name(a), (unsigned long long)r.act_dist[a]);
  printf("},\n \"cov\": {\"api\": %llu, \"req\": %llu, \"lreq\": %llu, \"objs\": %llu, \"api2\": %llu},\n",
         (unsigned long long)r.cov_api, (unsigned long long)r.cov_req, (unsigned long long)r.cov_lreq,
         (unsigned long long)r.cov_objs, (unsigned long long)r.cov_api2);
  printf(" \"branch\": [");
  for (int b = 0; b < KO_NBRANCH; b++) printf("%s%llu", b ? ", " : "", (unsigned long long)r.branch[b]);
  printf("],\n \"outdeg_hist\": {");
  int first = 1;
  for (int k = 0; k < 32; k++) if (r.outdeg_hist[k]) { printf("%s\"%d\": %llu", first ? "" : ", ", k, (unsigned long long)r.outdeg_hist[k]); first = 0; }
  printf("},\n \"level_width\": [");
  for (int l = 0; l < r.nlevels; l++) printf("%s%llu", l ? ", " : "", (unsigned long long)r.level_width[l]);
  printf("],\n \"err_kind\": %d, \"err_action\": \"%s\", \"err_self\": %d, \"err_invariant\": %d,"
         " \"err_level\": %d, \"trace_len\": %d}\n",
         r.err_kind, r.err_action >= 0 ? ko_action_name(r.err_action) : "", r.err_self,
         r.err_invariant, r.err_level, r.trace_len);
  if (print_trace && h) {
    size_t n = ko_trace_text(h, NULL, 0);
    char *buf = malloc(n + 1);
    ko_trace_text(h, buf, n + 1);
    fputs(buf, stderr);
    free(buf);
  }
  ko_free(h);
  return 0;
}

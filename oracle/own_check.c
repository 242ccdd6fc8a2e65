/* oracle/own_check.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Prints what GMAP's host code reads from the Dynprog_* entry points that are not DP fills: the
 * consistent-pair table behind Dynprog_consistent_p (dynprog.c:895) for every Mode_T and genestrand,
 * Dynprog_score (dynprog.c:126) over a grid of counts, defect rates and user penalties, and the limits of a
 * Dynprog_new handle (dynprog.c:631).  oracle/ref.mk links it twice: with the reference's own dynprog
 * objects (_ref/own_check_ref) and with the drop-in shim compiled -DGMAPDP_SHIM_OWN instead of them
 * (_ref/own_check_shim); tests/test_shim_own.py requires the two outputs to be identical.  Neither calls
 * the GPU.
 */
#ifdef HAVE_CONFIG_H
#include "config.h"
#endif
#include <stdio.h>
#include "bool.h"
#include "mode.h"
#include "dynprog.h"

int
main (void) {
  int mode, gs, c, g, m, n, k;
  static const double rates[] = {0.0, 0.0029, 0.003, 0.01, 0.014, 0.2};
  for (mode = STANDARD; mode <= TTOC_NONSTRANDED; mode++) {
    const int stranded = mode == STANDARD || mode == CMET_STRANDED || mode == ATOI_STRANDED || mode == TTOC_STRANDED;
    Dynprog_init((Mode_T) mode);
    for (gs = 0; gs < 3; gs++) {
      unsigned long h = 1469598103934665603UL, ones = 0;
      if (stranded ? gs != 0 : gs == 0) continue;  /* the reference allocates only these genestrands */
      for (c = 0; c < 128; c++)
        for (g = 0; g < 128; g++) {
          const int v = Dynprog_consistent_p(c, g, g, gs) ? 1 : 0;
          ones += v;
          h = (h ^ (unsigned long) (v + 2 * c + 1000 * g)) * 1099511628211UL;
        }
      printf("consistent mode %d genestrand %d: %lu pairs, digest %016lx\n", mode, gs, ones, h);
      /* g_alt: consistent through the alternate genome character only */
      for (c = 'A'; c <= 'z'; c += 7)
        printf(" %d", Dynprog_consistent_p(c, 'Q', 'G', gs) ? 1 : 0);
      printf("\n");
    }
    Dynprog_term((Mode_T) mode);
  }
  for (k = 0; k < 6; k++)
    for (m = 0; m < 3; m++)
      for (n = 0; n < 3; n++)
        printf("score %g %d %d: %d %d %d\n", rates[k], m, n,
               Dynprog_score(100 + 7 * m, 3 * n, m, 2 * n + m, n, m * n, rates[k], -9, -2, false),
               Dynprog_score(100 + 7 * m, 3 * n, m, 2 * n + m, n, m * n, rates[k], -9, -2, true),
               Dynprog_score(m, n, 3, 4, 5, 6, rates[k], -11, -1, k & 1));
  {
    static const int args[][5] = {{0, 0, 0, 0, 0}, {20, 10, 40, 10, 10}, {100, 10, 500, 80, 10}, {600, 5, 60, 10, 300},
                                   {1000, 10, 1000, 3000, 0}};
    for (k = 0; k < 5; k++) {
      Dynprog_T d = Dynprog_new(args[k][0], args[k][1], args[k][2], args[k][3], args[k][4], k & 1);
      printf("new %d: max_rlength %d max_glength %d\n", k, d->max_rlength, d->max_glength);
      Dynprog_free(&d);
      printf("freed %d: %s\n", k, d == NULL ? "NULL" : "not NULL");
    }
  }
  return 0;
}

/* oracle/fiber_check.c -- TEST INFRASTRUCTURE ONLY.
 *
 * The drop-in's worker fibers (gmap-2024_amd/shim, GMAPDP_SHIM_OWN: pthread_create / _join / _getspecific /
 * _setspecific wrapped) without a GPU: N "workers" created as GMAP creates them, each keeping its own value
 * under a pthread key (as except.c keeps its exception stack), recursing on its fiber stack, and returning a
 * value that pthread_join hands back.  oracle/ref.mk links it with the shim exactly as gmap_gpu_nosimd is
 * linked; tests/test_shim_own.py runs it with fibers on and off.  Prints one line: "fibers ok N".
 */
#include <pthread.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

static pthread_key_t key;

static long
depth (long n, volatile char *probe) {
  volatile char buf[512];
  buf[0] = (char) n;
  if (n == 0) return (long) (buf[0] + (probe != NULL));
  return depth(n - 1, buf) + 1;
}

static void *
worker (void *arg) {
  long id = (long) (intptr_t) arg, i, acc = 0;
  pthread_setspecific(key, (void *) (intptr_t) (id + 1));
  for (i = 0; i < 1000; i++) {
    if ((long) (intptr_t) pthread_getspecific(key) != id + 1) return (void *) (intptr_t) -1;
    acc += depth(200, NULL);  /* ~100 KB of stack */
  }
  return (void *) (intptr_t) (id * 7 + (acc == 1000L * 201L ? 0 : 100000));
}

int
main (int argc, char **argv) {
  int n = argc > 1 ? atoi(argv[1]) : 64, i, bad = 0;
  pthread_t *t = (pthread_t *) calloc((size_t) n, sizeof(pthread_t));
  pthread_key_create(&key, NULL);
  pthread_setspecific(key, (void *) (intptr_t) 4242);
  for (i = 0; i < n; i++) pthread_create(&t[i], NULL, worker, (void *) (intptr_t) i);
  for (i = 0; i < n; i++) {
    void *r = NULL;
    pthread_join(t[i], &r);
    if ((long) (intptr_t) r != 7L * i) bad++;
  }
  if ((long) (intptr_t) pthread_getspecific(key) != 4242) bad++;
  if (bad) {
    printf("fibers bad %d\n", bad);
    return 1;
  }
  printf("fibers ok %d\n", n);
  return 0;
}

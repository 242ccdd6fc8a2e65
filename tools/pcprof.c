/* Sampling PC profiler for the end-to-end runs (measurement tool, not product).
 *
 * Linked into the unstripped gmap_prof_V / gmap_gpu_prof_V programs (oracle/ref.mk); idle unless
 * PCPROF_OUT names an output file.  ITIMER_PROF ticks every PCPROF_US (default 1000) microseconds of
 * process CPU time and SIGPROF lands on the thread that used it; the handler records the interrupted
 * program counter and a thread role (0 GMAP's own threads, 1 the drop-in's fiber hosts, 2 its
 * dispatchers, 3 other named threads: HIP's).  At exit the samples and /proc/self/maps are written;
 * tools/pcprof.py resolves them to functions with nm.
 */
#define _GNU_SOURCE
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/time.h>
#include <ucontext.h>

static uint64_t *pc_samples;
static size_t pc_cap;
static size_t pc_n;
static const char *pc_out;

static void
pc_handler (int sig, siginfo_t *si, void *ucv) {
  ucontext_t *uc = (ucontext_t *) ucv;
  char name[16];
  uint64_t role = 0;
  size_t i;
  (void) sig;
  (void) si;
  i = __atomic_fetch_add(&pc_n, 1, __ATOMIC_RELAXED);
  if (i >= pc_cap) return;
  name[0] = '\0';
  prctl(PR_GET_NAME, name, 0, 0, 0);
  if (strncmp(name, "gmapdp-fibers", 13) == 0) role = 1;
  else if (strncmp(name, "gmapdp-q", 8) == 0) role = 2;
  else if (strncmp(name, "gmap", 4) != 0) role = 3;
  pc_samples[i] = ((uint64_t) uc->uc_mcontext.gregs[REG_RIP] & 0x00FFFFFFFFFFFFFFULL) | (role << 56);
}

static void
pc_dump (void) {
  struct itimerval off;
  FILE *f, *m;
  char line[4096];
  size_t i, n;
  memset(&off, 0, sizeof(off));
  setitimer(ITIMER_PROF, &off, NULL);
  n = __atomic_load_n(&pc_n, __ATOMIC_RELAXED);
  if (n > pc_cap) n = pc_cap;
  f = fopen(pc_out, "w");
  if (f == NULL) return;
  fprintf(f, "# pcprof samples=%zu period_us=%s\n", n, getenv("PCPROF_US") ? getenv("PCPROF_US") : "1000");
  m = fopen("/proc/self/maps", "r");
  while (m != NULL && fgets(line, sizeof(line), m) != NULL) fprintf(f, "M %s", line);
  if (m != NULL) fclose(m);
  for (i = 0; i < n; i++) fprintf(f, "S %llx\n", (unsigned long long) pc_samples[i]);
  fclose(f);
}

__attribute__((constructor)) static void
pc_start (void) {
  struct sigaction sa;
  struct itimerval it;
  long us;
  pc_out = getenv("PCPROF_OUT");
  if (pc_out == NULL || pc_out[0] == '\0') return;
  us = getenv("PCPROF_US") ? atol(getenv("PCPROF_US")) : 1000;
  if (us < 100) us = 100;
  pc_cap = (size_t) 1 << 24;
  pc_samples = (uint64_t *) calloc(pc_cap, sizeof(uint64_t));
  if (pc_samples == NULL) return;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = pc_handler;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, NULL);
  atexit(pc_dump);
  memset(&it, 0, sizeof(it));
  it.it_interval.tv_usec = us;
  it.it_value.tv_usec = us;
  setitimer(ITIMER_PROF, &it, NULL);
}

/* lastwords.c — bench.py's held line, written to stdout if the process is ended by a signal.
 *
 * bench.py secures its first multi-GPU line (the RCCL job, timed and verified) before the later,
 * optional phases run (the push gathers over IPC-mapped peer memory, the weak job, the
 * loopback).  A hang in those phases is bounded by bench.py's watchdog thread; a crash is not: a
 * GPU memory fault makes the HIP runtime abort() the process, and when any rank dies torchrun
 * ends the others with SIGTERM while they wait in a collective — in neither case does Python run
 * again.  This library keeps the serialized line in a static buffer and installs handlers for
 * SIGABRT, SIGSEGV, SIGBUS, SIGFPE, SIGILL and SIGTERM that write it to fd 1 (write(2) only:
 * async-signal-safe), once, then restore the previous disposition and re-raise the signal, so
 * the process still ends as it would have (exit status unchanged).
 *
 * Bench infrastructure, not the product: no GPU code, nothing from the aggregation library.
 *   gcc -O2 -fPIC -shared tools/lastwords.c -o tools/liblastwords.so
 */
#include <signal.h>
#include <stdatomic.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#define LW_CAP (1 << 18)

static char lw_buf[2][LW_CAP];
static size_t lw_len[2];
static atomic_int lw_cur = -1;   /* the buffer that holds the line, or -1: nothing to write */
static atomic_int lw_done = 0;   /* written once */
static struct sigaction lw_old[NSIG];
static int lw_installed = 0;
static const int lw_sigs[] = {SIGABRT, SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGTERM};

static void lw_write_all(const char* p, size_t n) {
  while (n > 0) {
    const ssize_t k = write(1, p, n);
    if (k <= 0) return;
    p += k;
    n -= (size_t)k;
  }
}

static void lw_handler(int sig) {
  const int cur = atomic_load(&lw_cur);
  if (cur >= 0 && !atomic_exchange(&lw_done, 1)) lw_write_all(lw_buf[cur], lw_len[cur]);
  sigaction(sig, &lw_old[sig], NULL);
  raise(sig);
}

static int lw_install(void) {
  if (lw_installed) return 0;
  for (size_t i = 0; i < sizeof lw_sigs / sizeof lw_sigs[0]; ++i) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = lw_handler;
    sigemptyset(&sa.sa_mask);
    if (sigaction(lw_sigs[i], &sa, &lw_old[lw_sigs[i]]) != 0) return -2;
  }
  lw_installed = 1;
  return 0;
}

/* Hold `line` (n bytes; a trailing newline is added): written if a handled signal ends the
 * process before lw_clear().  Double-buffered: a signal during the update writes the previous
 * line whole.  0, or -1 if the line does not fit, -2 if the handlers cannot be installed. */
int lw_set(const char* line, int64_t n) {
  if (!line || n < 0 || n + 1 > LW_CAP) return -1;
  const int rc = lw_install();
  if (rc) return rc;
  const int next = atomic_load(&lw_cur) == 0 ? 1 : 0;
  memcpy(lw_buf[next], line, (size_t)n);
  lw_buf[next][n] = '\n';
  lw_len[next] = (size_t)n + 1;
  atomic_store(&lw_cur, next);
  return 0;
}

/* Nothing to write any more (the line was printed normally).  The handlers stay installed and
 * just pass the signal on. */
int lw_clear(void) {
  atomic_store(&lw_cur, -1);
  return 0;
}

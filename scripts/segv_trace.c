/* segv_trace.c — diagnostic: on SIGSEGV / SIGABRT print the native backtrace (each frame's library and
 * offset, dladdr via backtrace_symbols_fd) and the loaded-library map to stderr, then re-raise.
 * Loaded by bench.py when LMM_SEGV_TRACE=1 (ctypes.CDLL: the constructor installs the handlers), to find
 * which library owns the frames of an exit-time crash.  Host code only; no GPU calls.
 * Build: gcc -O1 -g -shared -fPIC scripts/segv_trace.c -o scripts/libsegv_trace.so */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void put(const char* s) { (void)!write(2, s, strlen(s)); }

static void handler(int sig, siginfo_t* si, void* uc) {
  (void)uc;
  void* fr[64];
  char buf[64];
  put(sig == SIGSEGV ? "\n[segv_trace] SIGSEGV, fault address " : "\n[segv_trace] SIGABRT ");
  if (sig == SIGSEGV) {
    unsigned long a = (unsigned long)si->si_addr;
    char* p = buf + sizeof buf - 1;
    *p = 0;
    do {
      *--p = "0123456789abcdef"[a & 15];
      a >>= 4;
    } while (a && p > buf + 2);
    *--p = 'x';
    *--p = '0';
    put(p);
  }
  put("\n[segv_trace] backtrace (library(+offset) [address]):\n");
  int n = backtrace(fr, 64);
  backtrace_symbols_fd(fr, n, 2);
  put("[segv_trace] /proc/self/maps (executable mappings):\n");
  int fd = open("/proc/self/maps", O_RDONLY);
  if (fd >= 0) {
    char line[512];
    int len = 0;
    char c;
    while (read(fd, &c, 1) == 1) {
      if (len < (int)sizeof line - 1)
        line[len++] = c;
      if (c == '\n') {
        line[len] = 0;
        if (strstr(line, " r-xp ") || strstr(line, " r-xs "))
          put(line);
        len = 0;
      }
    }
    close(fd);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((constructor)) static void install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGABRT, &sa, 0);
}

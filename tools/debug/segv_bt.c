// SIGSEGV / SIGBUS handler that prints the native backtrace (with the faulting address) to stderr,
// then re-raises with the default action. Load with ctypes and call segv_bt_install() before the
// code under test (pytest -p no:faulthandler, so this handler is the one installed).
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>
#include <ucontext.h>
#include <stdlib.h>
#include <sys/resource.h>

static void handler(int sig, siginfo_t* si, void* uc_) {
  char buf[128];
  ucontext_t* uc = (ucontext_t*)uc_;
  struct rlimit rl;
  getrlimit(RLIMIT_STACK, &rl);
  int n = snprintf(buf, sizeof buf, "\n[segv_bt] signal %d addr %p rip %p rsp %p stack-rlimit %lld\n", sig,
                   si->si_addr, (void*)uc->uc_mcontext.gregs[REG_RIP], (void*)uc->uc_mcontext.gregs[REG_RSP],
                   (long long)rl.rlim_cur);
  write(2, buf, n);
  void* frames[64];
  int k = backtrace(frames, 64);
  backtrace_symbols_fd(frames, k, 2);
  FILE* f = fopen("/proc/self/maps", "r");
  if (f) {  // the mappings, to resolve library offsets afterwards
    char line[512];
    while (fgets(line, sizeof line, f))
      if (strstr(line, "r-xp")) write(2, line, strlen(line));
    fclose(f);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

// Every thread that may fault needs its own alternate stack (a stack overflow leaves no room for the
// handler on the thread's stack): installed here for the calling thread; other threads fall back to
// their own stack.
void segv_bt_install(void) {
  stack_t ss;
  ss.ss_sp = malloc(1 << 20);
  ss.ss_size = 1 << 20;
  ss.ss_flags = 0;
  sigaltstack(&ss, 0);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = handler;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigaction(SIGSEGV, &sa, 0);
  sigaction(SIGBUS, &sa, 0);
}

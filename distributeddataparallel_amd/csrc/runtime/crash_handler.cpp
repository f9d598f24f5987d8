// Native crash reporter: on SIGSEGV/SIGBUS/SIGFPE/SIGILL/SIGABRT print the native backtrace
// (demangled, with the owning shared object) to stderr, then hand the signal to the previous
// handler (Python's faulthandler prints the Python frames after us). Enabled by
// XDDP_NATIVE_BACKTRACE=1 or distributeddataparallel_amd.utils.debug.install_crash_handler().
// Failure-detection counterpart of the reference stack's C++ stack dumps on watchdog errors
// (SURVEY.md §5.3).
#include <cxxabi.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace xddp {

namespace {

constexpr int kSigs[] = {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT};
struct sigaction g_prev[sizeof(kSigs) / sizeof(kSigs[0])];
volatile sig_atomic_t g_in_handler = 0;

void write_str(const char* s) { (void)!write(STDERR_FILENO, s, strlen(s)); }

void handler(int sig, siginfo_t* info, void* uctx) {
  if (!g_in_handler) {
    g_in_handler = 1;
    char buf[512];
    snprintf(buf, sizeof(buf), "\n[xddp] fatal signal %d (%s) at address %p, pid %d; native backtrace:\n", sig,
             strsignal(sig), info ? info->si_addr : nullptr, (int)getpid());
    write_str(buf);
    void* frames[64];
    const int n = backtrace(frames, 64);
    for (int i = 1; i < n; ++i) {  // frame 0 is this handler
      Dl_info di;
      const char* obj = "?";
      const char* sym = nullptr;
      uintptr_t off = 0;
      if (dladdr(frames[i], &di)) {
        obj = di.dli_fname ? di.dli_fname : "?";
        sym = di.dli_sname;
        off = di.dli_saddr ? (uintptr_t)frames[i] - (uintptr_t)di.dli_saddr
                           : (uintptr_t)frames[i] - (uintptr_t)di.dli_fbase;
      }
      int st = -1;
      char* dem = sym ? abi::__cxa_demangle(sym, nullptr, nullptr, &st) : nullptr;  // not async-safe; best effort
      const char* slash = strrchr(obj, '/');
      snprintf(buf, sizeof(buf), "  #%-2d %s+0x%lx  (%s)\n", i, dem ? dem : (sym ? sym : "??"), (unsigned long)off,
               slash ? slash + 1 : obj);
      write_str(buf);
      free(dem);
    }
  }
  // chain to the previous disposition (e.g. Python faulthandler), else default + re-raise
  for (size_t k = 0; k < sizeof(kSigs) / sizeof(kSigs[0]); ++k) {
    if (kSigs[k] != sig) continue;
    const struct sigaction& p = g_prev[k];
    if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction) {
      p.sa_sigaction(sig, info, uctx);
      return;
    }
    if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
      p.sa_handler(sig);
      return;
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

bool install_crash_handler() {
  static bool installed = false;
  if (installed) return false;
  void* warm[2];
  backtrace(warm, 2);  // loads libgcc's unwinder now, not inside the signal handler
  for (size_t k = 0; k < sizeof(kSigs) / sizeof(kSigs[0]); ++k) {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kSigs[k], &sa, &g_prev[k]);
  }
  installed = true;
  return true;
}

}  // namespace xddp

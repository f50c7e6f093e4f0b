// crash_maps.cpp -- diagnostic SIGSEGV / SIGBUS / SIGILL / SIGFPE report (az_diag_crash_report): on a
// fault in ANY thread of the process, append to a file the faulting thread's id and name
// (/proc/thread-self/comm: the engine names its host threads az-gamma / az-noise-pf), the fault
// address, the PC and a copy of /proc/self/maps, so a crash inside a profiler run can be
// symbolised afterwards (which library holds the PC and the thread's frames).  Then the previous
// handler (e.g. rocprofv3's glog failure handler, which prints the frames) runs as before.
// Async-signal-safe: open / read / write / close only, no allocation, no stdio.
#include <fcntl.h>
#include <signal.h>
#include <string.h>
#include <sys/syscall.h>
#include <ucontext.h>
#include <unistd.h>

namespace {

char g_path[512];
struct sigaction g_old[32];
const int kSignals[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE};

void put(int fd, const char* s) { (void)!write(fd, s, strlen(s)); }

void put_hex(int fd, unsigned long v) {
    char b[19] = "0x";
    for (int i = 0; i < 16; ++i) b[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 15];
    b[18] = 0;
    put(fd, b);
}

void put_dec(int fd, long v) {
    char b[24];
    int n = 0;
    if (v < 0) { put(fd, "-"); v = -v; }
    do { b[n++] = (char)('0' + v % 10); v /= 10; } while (v && n < 23);
    char o[24];
    for (int i = 0; i < n; ++i) o[i] = b[n - 1 - i];
    o[n] = 0;
    put(fd, o);
}

void copy_file(int out, const char* path) {
    const int in = open(path, O_RDONLY);
    if (in < 0) return;
    char buf[4096];
    for (;;) {
        const ssize_t k = read(in, buf, sizeof buf);
        if (k <= 0) break;
        (void)!write(out, buf, (size_t)k);
    }
    close(in);
}

void handler(int sig, siginfo_t* si, void* uc) {
    const int fd = open(g_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd >= 0) {
        put(fd, "=== az crash report: signal ");
        put_dec(fd, sig);
        put(fd, " pid ");
        put_dec(fd, (long)getpid());
        put(fd, " tid ");
        put_dec(fd, (long)syscall(SYS_gettid));
        put(fd, " thread name: ");
        copy_file(fd, "/proc/thread-self/comm");   // ends with a newline
        put(fd, "fault address ");
        put_hex(fd, (unsigned long)si->si_addr);
        put(fd, " code ");
        put_dec(fd, si->si_code);
#if defined(__x86_64__)
        const ucontext_t* u = static_cast<const ucontext_t*>(uc);
        put(fd, " pc ");
        put_hex(fd, (unsigned long)u->uc_mcontext.gregs[REG_RIP]);
        put(fd, " sp ");
        put_hex(fd, (unsigned long)u->uc_mcontext.gregs[REG_RSP]);
#endif
        put(fd, "\n--- /proc/self/maps\n");
        copy_file(fd, "/proc/self/maps");
        put(fd, "--- /proc/self/task/*/comm: see the thread name above; end of report\n");
        close(fd);
    }
    // the previous disposition runs on the re-executed fault (or directly for a default one)
    sigaction(sig, &g_old[sig], nullptr);
    if (g_old[sig].sa_handler == SIG_DFL || g_old[sig].sa_handler == SIG_IGN) raise(sig);
}

}  // namespace

extern "C" int az_diag_crash_report(const char* path) {
    if (!path || strlen(path) >= sizeof g_path) return -1;
    strcpy(g_path, path);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    for (int s : kSignals)
        if (sigaction(s, &sa, &g_old[s]) != 0) return -1;
    return 0;
}

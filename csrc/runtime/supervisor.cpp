// Process supervisor for the local ElasticOperator.
//
// Replaces the reference's implied Go/Kubernetes pod lifecycle
// (reference .pre-commit-config.yaml:42-49, docs/design/elastic-training-operator.md)
// with a node-local native supervisor:
//   * spawn: fork + execve with a prepared environment, its own process group
//     (so a role and all its children are signalled together), CPU affinity
//     (sched_setaffinity) from the resource plan, PR_SET_PDEATHSIG so nothing
//     outlives the operator, stdout/stderr appended to a per-role log file;
//   * exit events: every child gets a pidfd registered in one epoll set, so
//     edl_sup_wait() returns {pid, exit code | signal, timestamp} within
//     microseconds of a crash / OOM-kill / kill -9 (the TTR "detect" phase);
//     no polling interval, no SIGCHLD handler in the (threaded) Python host;
//   * kill / group kill for SIGTERM -> SIGKILL escalation (driven by Python).
// Everything the child does between fork and exec is async-signal-safe:
// argv/envp/cpu sets/log fd are prepared before fork.
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#ifndef SYS_pidfd_open
#define SYS_pidfd_open 434
#endif
#ifndef P_PIDFD
#define P_PIDFD 3
#endif

namespace {

struct Child {
  pid_t pid;
  int pidfd;
  std::string name;
};

struct Supervisor {
  int epfd = -1;
  std::mutex mu;
  std::map<pid_t, Child> children;  // live (not yet reaped)
  std::map<int, pid_t> fd2pid;
};

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

}  // namespace

extern "C" {

struct EdlExitEvent {
  int32_t pid;
  int32_t exit_code;  // valid when signal == 0
  int32_t signal;     // terminating signal or 0
  int32_t core;       // core dumped
  int64_t ts_ns;      // wall clock when reaped
};

void* edl_sup_create() {
  auto* s = new Supervisor();
  s->epfd = epoll_create1(EPOLL_CLOEXEC);
  if (s->epfd < 0) {
    delete s;
    return nullptr;
  }
  return s;
}

// argv / envp: NULL-terminated arrays.  cpus: array of ncpus CPU ids (may be 0).
// Returns 0 and writes *pid_out, or -errno.
int edl_sup_spawn(void* h, const char* name, const char* const* argv, const char* const* envp, const char* cwd,
                  const char* log_path, const int* cpus, int ncpus, int new_pgrp, int* pid_out) {
  auto* s = static_cast<Supervisor*>(h);
  if (!s || !argv || !argv[0]) return -EINVAL;
  int logfd = -1;
  if (log_path && *log_path) {
    logfd = open(log_path, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (logfd < 0) return -errno;
  }
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int i = 0; i < ncpus; ++i)
    if (cpus[i] >= 0 && cpus[i] < CPU_SETSIZE) CPU_SET(cpus[i], &set);
  const pid_t parent = getpid();
  int errpipe[2];
  if (pipe2(errpipe, O_CLOEXEC) != 0) {
    if (logfd >= 0) close(logfd);
    return -errno;
  }
  pid_t pid = fork();
  if (pid < 0) {
    int e = errno;
    close(errpipe[0]);
    close(errpipe[1]);
    if (logfd >= 0) close(logfd);
    return -e;
  }
  if (pid == 0) {
    // ---- child: async-signal-safe only ----
    close(errpipe[0]);
    if (new_pgrp) setpgid(0, 0);
    prctl(PR_SET_PDEATHSIG, SIGKILL);
    if (getppid() != parent) _exit(127);  // parent already gone
    sigset_t none;
    sigemptyset(&none);
    sigprocmask(SIG_SETMASK, &none, nullptr);
    if (ncpus > 0) sched_setaffinity(0, sizeof(set), &set);
    if (logfd >= 0) {
      dup2(logfd, 1);
      dup2(logfd, 2);
    }
    if (cwd && *cwd && chdir(cwd) != 0) {
      int e = errno;
      (void)!write(errpipe[1], &e, sizeof(e));
      _exit(127);
    }
    if (envp)
      execve(argv[0], (char* const*)argv, (char* const*)envp);
    else
      execv(argv[0], (char* const*)argv);
    int e = errno;
    (void)!write(errpipe[1], &e, sizeof(e));
    _exit(127);
  }
  // ---- parent ----
  close(errpipe[1]);
  if (logfd >= 0) close(logfd);
  if (new_pgrp) setpgid(pid, pid);  // avoid the race with the child's own setpgid
  int child_err = 0;
  ssize_t n = read(errpipe[0], &child_err, sizeof(child_err));
  close(errpipe[0]);
  if (n == (ssize_t)sizeof(child_err)) {  // exec failed: reap and report
    waitpid(pid, nullptr, 0);
    return -child_err;
  }
  int pidfd = (int)syscall(SYS_pidfd_open, pid, 0);
  {
    std::lock_guard<std::mutex> g(s->mu);
    s->children[pid] = Child{pid, pidfd, name ? name : ""};
    if (pidfd >= 0) {
      epoll_event ev{};
      ev.events = EPOLLIN;
      ev.data.fd = pidfd;
      epoll_ctl(s->epfd, EPOLL_CTL_ADD, pidfd, &ev);
      s->fd2pid[pidfd] = pid;
    }
  }
  *pid_out = pid;
  return 0;
}

static int reap(Supervisor* s, pid_t pid, EdlExitEvent* out) {
  int status = 0;
  pid_t r = waitpid(pid, &status, WNOHANG);
  if (r != pid) return 0;
  out->pid = pid;
  out->exit_code = WIFEXITED(status) ? WEXITSTATUS(status) : -1;
  out->signal = WIFSIGNALED(status) ? WTERMSIG(status) : 0;
  out->core = WIFSIGNALED(status) ? (WCOREDUMP(status) ? 1 : 0) : 0;
  out->ts_ns = now_ns();
  auto it = s->children.find(pid);
  if (it != s->children.end()) {
    if (it->second.pidfd >= 0) {
      epoll_ctl(s->epfd, EPOLL_CTL_DEL, it->second.pidfd, nullptr);
      s->fd2pid.erase(it->second.pidfd);
      close(it->second.pidfd);
    }
    s->children.erase(it);
  }
  return 1;
}

// Wait up to timeout_ms for exits; fills at most max events; returns the count (or -errno).
int edl_sup_wait(void* h, int timeout_ms, EdlExitEvent* out, int max) {
  auto* s = static_cast<Supervisor*>(h);
  if (!s || max <= 0) return -EINVAL;
  int count = 0;
  {
    // children without a pidfd (very old kernels) are checked every call
    std::lock_guard<std::mutex> g(s->mu);
    std::vector<pid_t> nofd;
    for (auto& kv : s->children)
      if (kv.second.pidfd < 0) nofd.push_back(kv.first);
    for (pid_t p : nofd)
      if (count < max) count += reap(s, p, &out[count]);
  }
  if (count > 0) return count;
  epoll_event evs[64];
  int n = epoll_wait(s->epfd, evs, 64, timeout_ms);
  if (n < 0) return errno == EINTR ? 0 : -errno;
  std::lock_guard<std::mutex> g(s->mu);
  for (int i = 0; i < n && count < max; ++i) {
    auto it = s->fd2pid.find(evs[i].data.fd);
    if (it == s->fd2pid.end()) continue;
    count += reap(s, it->second, &out[count]);
  }
  return count;
}

// Children that are being torn down right now (PF_EXITING set in
// /proc/<pid>/stat flags) but not yet reaped.  A SIGKILLed process with a
// large address space (hundreds of GB of GPU + shared memory mappings) takes
// seconds to unmap before its pidfd becomes readable; its PF_EXITING flag is
// set at the start of do_exit(), so this reports the death seconds earlier.
int edl_sup_exiting(void* h, int* pids, int max) {
  auto* s = static_cast<Supervisor*>(h);
  std::vector<pid_t> live;
  {
    std::lock_guard<std::mutex> g(s->mu);
    for (auto& kv : s->children) live.push_back(kv.first);
  }
  int n = 0;
  char path[64], buf[1024];
  for (pid_t p : live) {
    if (n >= max) break;
    snprintf(path, sizeof(path), "/proc/%d/stat", (int)p);
    int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;
    ssize_t r = read(fd, buf, sizeof(buf) - 1);
    close(fd);
    if (r <= 0) continue;
    buf[r] = 0;
    // fields after "(comm)": state ppid pgrp session tty_nr tpgid flags ...
    char* rp = strrchr(buf, ')');
    if (!rp) continue;
    char state = 0;
    long ppid, pgrp, sess, tty, tpgid;
    unsigned long flags = 0;
    if (sscanf(rp + 2, "%c %ld %ld %ld %ld %ld %lu", &state, &ppid, &pgrp, &sess, &tty, &tpgid, &flags) != 7)
      continue;
    if ((flags & 0x4UL) || state == 'Z' || state == 'X') pids[n++] = (int)p;  // PF_EXITING
  }
  return n;
}

int edl_sup_kill(void* h, int pid, int sig, int group) {
  (void)h;
  int r = group ? kill(-pid, sig) : kill(pid, sig);
  return r == 0 ? 0 : -errno;
}

int edl_sup_num_children(void* h) {
  auto* s = static_cast<Supervisor*>(h);
  std::lock_guard<std::mutex> g(s->mu);
  return (int)s->children.size();
}

void edl_sup_destroy(void* h) {
  auto* s = static_cast<Supervisor*>(h);
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(s->mu);
    for (auto& kv : s->children) {
      kill(-kv.first, SIGKILL);
      kill(kv.first, SIGKILL);
    }
  }
  for (int i = 0; i < 100; ++i) {
    EdlExitEvent ev[16];
    if (edl_sup_num_children(s) == 0) break;
    edl_sup_wait(s, 20, ev, 16);
  }
  {
    std::lock_guard<std::mutex> g(s->mu);
    for (auto& kv : s->children)
      if (kv.second.pidfd >= 0) close(kv.second.pidfd);
    close(s->epfd);
    s->children.clear();
  }  // the lock must be released before the supervisor (and its mutex) is freed
  delete s;
}

}  // extern "C"

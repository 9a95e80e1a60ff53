// Host-side self-test of the native runtime (csrc/runtime/supervisor.cpp,
// shm_store.cpp), built by tests/test_native_sanitizers.py with
// -fsanitize=address,undefined and separately with -fsanitize=thread
// (SURVEY.md §4.2 tier T1, §5.2).  No GPU: only the host paths — process
// supervision (spawn, exit events from pidfd/epoll, kill, concurrent waiters)
// and the A/B shared-memory checkpoint store (begin/commit/latest, torn-write
// invisibility, concurrent readers while a writer flips slots).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <signal.h>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

extern "C" {
struct EdlExitEvent {
  int32_t pid, exit_code, signal, core;
  int64_t ts_ns;
};
void* edl_sup_create();
int edl_sup_spawn(void*, const char*, const char* const*, const char* const*, const char*, const char*, const int*, int,
                  int, int*);
int edl_sup_wait(void*, int, EdlExitEvent*, int);
int edl_sup_kill(void*, int, int, int);
int edl_sup_num_children(void*);
void edl_sup_destroy(void*);
void* edl_shm_open(const char*, uint64_t, int, int);
void* edl_shm_data(void*, int);
int edl_shm_begin(void*);
int edl_shm_commit(void*, int, int64_t, int64_t, uint64_t, uint64_t, const char*);
int edl_shm_latest(void*, int64_t*, int64_t*, uint64_t*, uint64_t*, char*, int);
int edl_shm_close(void*, int);
int edl_shm_populate_async(void*, int);
uint64_t edl_shm_populate_progress(void*, uint64_t*);
}

#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                       \
    }                                                                \
  } while (0)

static int collect(void* sup, std::vector<EdlExitEvent>& out, size_t want, int budget_ms) {
  EdlExitEvent ev[8];
  while (out.size() < want && budget_ms > 0) {
    int n = edl_sup_wait(sup, 50, ev, 8);
    CHECK(n >= 0);
    for (int i = 0; i < n; ++i) out.push_back(ev[i]);
    budget_ms -= 50;
  }
  return (int)out.size();
}

static void test_supervisor() {
  void* sup = edl_sup_create();
  CHECK(sup);
  const char* env[] = {"EDL_TEST=1", nullptr};
  const char* ok_argv[] = {"/bin/sh", "-c", "exit 3", nullptr};
  const char* sleep_argv[] = {"/bin/sleep", "30", nullptr};
  int p1 = 0, p2 = 0, p3 = 0;
  CHECK(edl_sup_spawn(sup, "t-ok", ok_argv, env, "/", "", nullptr, 0, 1, &p1) == 0);
  CHECK(edl_sup_spawn(sup, "t-sleep", sleep_argv, env, "/", "", nullptr, 0, 1, &p2) == 0);
  int cpu0 = 0;
  CHECK(edl_sup_spawn(sup, "t-pinned", ok_argv, env, "/", "/dev/null", &cpu0, 1, 1, &p3) == 0);
  std::vector<EdlExitEvent> got;
  collect(sup, got, 2, 5000);
  CHECK(got.size() == 2);
  for (auto& e : got) CHECK(e.exit_code == 3 && e.signal == 0 && (e.pid == p1 || e.pid == p3));
  CHECK(edl_sup_num_children(sup) == 1);
  CHECK(edl_sup_kill(sup, p2, SIGKILL, 1) == 0);
  got.clear();
  collect(sup, got, 1, 5000);
  CHECK(got.size() == 1 && got[0].pid == p2 && got[0].signal == SIGKILL);
  // many short children reaped by two concurrent waiters (event loop under TSan)
  const int N = 24;
  for (int i = 0; i < N; ++i) {
    int pid;
    CHECK(edl_sup_spawn(sup, "t-burst", ok_argv, env, "/", "", nullptr, 0, 1, &pid) == 0);
  }
  std::atomic<int> seen{0};
  auto waiter = [&] {
    EdlExitEvent ev[4];
    for (int k = 0; k < 200 && seen.load() < N; ++k) {
      int n = edl_sup_wait(sup, 20, ev, 4);
      if (n > 0) seen += n;
    }
  };
  std::thread a(waiter), b(waiter);
  a.join();
  b.join();
  CHECK(seen.load() == N);
  CHECK(edl_sup_num_children(sup) == 0);
  const char* bad_argv[] = {"/nonexistent/binary", nullptr};
  int pb = 0;
  int rc = edl_sup_spawn(sup, "t-bad", bad_argv, env, "/", "", nullptr, 0, 1, &pb);
  if (rc == 0) {  // exec failure is reported as an exit of the child
    got.clear();
    collect(sup, got, 1, 5000);
    CHECK(got.size() == 1 && got[0].exit_code != 0);
  }
  edl_sup_destroy(sup);
}

static void test_shm_store() {
  std::string name = "/edl-selftest-" + std::to_string(getpid());
  const uint64_t bytes = 1 << 20;
  void* w = edl_shm_open(name.c_str(), bytes, 2, 1);
  CHECK(w);
  int64_t step, epoch;
  uint64_t nb, cs;
  char meta[256];
  CHECK(edl_shm_latest(w, &step, &epoch, &nb, &cs, meta, sizeof(meta)) == -1);
  void* r = edl_shm_open(name.c_str(), 0, 0, 0);
  CHECK(r);
  std::atomic<bool> stop{false};
  std::atomic<int> reads{0};
  // reader: a committed slot is never the one being written, and its payload matches its step
  std::thread reader([&] {
    char m[256];
    while (!stop.load()) {
      int64_t s, e;
      uint64_t n, c;
      int slot = edl_shm_latest(r, &s, &e, &n, &c, m, sizeof(m));
      if (slot < 0) continue;
      // seqlock-style: trust a read only if the same slot still holds the same step
      // afterwards (the writer may be two commits ahead and rewriting this slot)
      int64_t s2, e2;
      uint64_t n2, c2;
      char m2[256];
      if (edl_shm_latest(r, &s2, &e2, &n2, &c2, m2, sizeof(m2)) != slot || s2 != s) continue;
      CHECK(c == (uint64_t)s * 7 + 1);
      CHECK(std::string(m) == "step=" + std::to_string(s));
      ++reads;
    }
  });
  for (int64_t s = 1; s <= 400; ++s) {
    int slot = edl_shm_begin(w);
    CHECK(slot == 0 || slot == 1);
    auto* p = static_cast<uint64_t*>(edl_shm_data(w, slot));
    for (uint64_t i = 0; i < bytes / 8; i += 512) p[i] = (uint64_t)s;
    std::string m = "step=" + std::to_string(s);
    CHECK(edl_shm_commit(w, slot, s, 1, bytes, (uint64_t)s * 7 + 1, m.c_str()) == 0);
  }
  stop = true;
  reader.join();
  // background population racing the writer and the reader's mapping, then a close that
  // must join the populating threads (one started, one cut short by close)
  CHECK(edl_shm_populate_async(w, 3) == 0 && edl_shm_populate_async(w, 3) == -1);
  for (int64_t s = 401; s <= 420; ++s) {
    int slot = edl_shm_begin(w);
    auto* p = static_cast<uint64_t*>(edl_shm_data(w, slot));
    for (uint64_t i = 0; i < bytes / 8; i += 512) p[i] = (uint64_t)s;
    CHECK(edl_shm_commit(w, slot, s, 1, bytes, (uint64_t)s * 7 + 1, ("step=" + std::to_string(s)).c_str()) == 0);
  }
  uint64_t total = 0, done = 0;
  for (int i = 0; i < 5000 && (done = edl_shm_populate_progress(w, &total)) < total; ++i) usleep(1000);
  CHECK(total >= 2 * bytes && done >= total);   // slots are rounded up to 2 MiB
  CHECK(edl_shm_populate_async(r, 2) == 0);   // closed below while (maybe) still running
  CHECK(edl_shm_latest(r, &step, &epoch, &nb, &cs, meta, sizeof(meta)) >= 0 && step == 420);
  CHECK(edl_shm_commit(w, 5, 1, 1, 8, 0, "") != 0);       // bad slot
  CHECK(edl_shm_commit(w, 0, 1, 1, bytes << 20, 0, "") != 0);  // larger than a slot
  edl_shm_close(r, 0);
  edl_shm_close(w, 1);
  printf("shm reads during writes: %d\n", reads.load());
}

int main() {
  test_supervisor();
  test_shm_store();
  printf("runtime selftest OK\n");
  return 0;
}

// How long does the kernel take to tear down a SIGKILLed process that maps a large snapshot segment?
// (no-survivor TTR: the operator hands the GPU to the standby only after the dead worker is reaped)
// modes: none | touch_read | populate_write | memcpy | pin (hipHostRegister) | populate_write_unmap
// usage: exit_cost_probe <mode> <GiB>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static void par(uint8_t* p, uint64_t n, int threads, int advice) {
  std::vector<std::thread> ts;
  uint64_t per = (n / threads + 4095) & ~4095ull;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([=] {
      uint64_t lo = per * t;
      if (lo >= n) return;
      uint64_t len = lo + per > n ? n - lo : per;
      if (advice) madvise(p + lo, len, advice);
      else memset(p + lo, 1, len);
    });
  for (auto& t : ts) t.join();
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  const std::string mode = argv[1];
  const uint64_t bytes = (uint64_t)atoll(argv[2]) << 30;
  const char* name = "/edl-exitprobe";
  shm_unlink(name);
  int fd = shm_open(name, O_RDWR | O_CREAT, 0600);
  if (fd < 0 || ftruncate(fd, bytes) != 0) return 3;
  // the file's pages exist before the child runs (a long-running job's segment is fully written)
  {
    uint8_t* p = (uint8_t*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    double t0 = now();
    par(p, bytes, 16, MADV_POPULATE_WRITE);
    printf("prefill %.2f s\n", now() - t0);
    munmap(p, bytes);
  }
  int pfd[2];
  if (pipe(pfd) != 0) return 4;
  pid_t pid = fork();
  if (pid == 0) {
    uint8_t* p = (uint8_t*)mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    double t0 = now();
    if (mode == "touch_read") par(p, bytes, 16, MADV_POPULATE_READ);
    if (mode == "populate_write" || mode == "populate_write_unmap") par(p, bytes, 16, MADV_POPULATE_WRITE);
    if (mode == "memcpy") par(p, bytes, 16, 0);
    if (mode == "gpu_memcpy") {  // a GPU context (and VRAM) plus a populated mapping
      void* d = nullptr;
      hipMalloc(&d, 1ull << 30);
      par(p, bytes, 16, 0);
    }
    if (mode == "pin") {
      hipError_t e = hipHostRegister(p, bytes, hipHostRegisterPortable);
      if (e != hipSuccess) fprintf(stderr, "hipHostRegister %d\n", (int)e);
    }
    double t1 = now();
    if (mode == "populate_write_unmap") munmap(p, bytes);
    double t2 = now();
    char msg[128];
    int n = snprintf(msg, sizeof msg, "%.2f %.2f", t1 - t0, t2 - t1);
    if (write(pfd[1], msg, n) != n) _exit(5);
    for (;;) pause();
  }
  char buf[128] = {0};
  if (read(pfd[0], buf, sizeof buf - 1) <= 0) return 6;
  // the KFD process entry of the child: it disappears when the driver has torn down the
  // child's GPU queues, which may be long before the kernel has reaped the process
  char kfd[96];
  snprintf(kfd, sizeof kfd, "/sys/class/kfd/kfd/proc/%d", (int)pid);
  const bool had_kfd = access(kfd, F_OK) == 0;
  double t0 = now(), t_kfd = -1;
  kill(pid, SIGKILL);
  int st;
  for (;;) {
    if (t_kfd < 0 && had_kfd && access(kfd, F_OK) != 0) t_kfd = now() - t0;
    if (waitpid(pid, &st, WNOHANG) == pid) break;
    usleep(500);
  }
  double t1 = now();
  if (had_kfd && t_kfd < 0) t_kfd = t1 - t0;
  printf("mode=%s gib=%lu setup/unmap_s=%s exit_s=%.3f kfd_entry=%d kfd_gone_s=%.3f\n", mode.c_str(), bytes >> 30, buf,
         t1 - t0, (int)had_kfd, t_kfd);
  shm_unlink(name);
  return 0;
}

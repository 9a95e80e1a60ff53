// Shared-memory checkpoint store + asynchronous D2H snapshot engine
// (SURVEY.md §2.4 N10, §3 CS7, §5.4).
//
// Segment  /dev/shm/<name>  (owned by the operator, so it survives worker death):
//   [SegHdr 4 KiB][SlotHdr x nslots, 4 KiB each][slot 0 data][slot 1 data]...
// Slots are A/B double-buffered: a snapshot always writes the slot that is NOT
// current, then publishes {step, epoch, nbytes, checksum, meta} in the slot
// header, sets state=COMMITTED and finally flips `current` — a writer that
// dies mid-copy leaves the previous committed slot untouched (torn-write
// safe).  Slot data is page-locked with hipHostRegister so the copies run as
// SDMA transfers at PCIe rate.
//
// Snapshot engine: a low-priority HIP stream per device.  A snapshot records
// an event on the caller's compute stream, makes the side stream wait on it,
// enqueues chunked hipMemcpyAsync D2H copies into the free slot and records a
// completion event; a committer thread waits for that event and publishes the
// slot.  The caller makes its NEXT optimizer step wait on the completion
// event (edl_ckpt_fence), so the copy overlaps forward/backward and never
// reads a half-updated parameter.
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint64_t kHdr = 4096;
constexpr uint32_t kEmpty = 0, kWriting = 1, kCommitted = 2;

struct SegHdr {
  char magic[8];
  uint64_t version;
  uint64_t slot_bytes;
  uint32_t nslots;
  int32_t current;  // committed slot or -1
  uint64_t gen;     // incremented on every commit
};

struct SlotHdr {
  uint64_t seq;
  int64_t step;
  int64_t epoch;
  uint64_t nbytes;
  uint64_t checksum;
  int64_t ts_ns;
  uint32_t state;
  uint32_t pad;
  char meta[4096 - 56];
};
static_assert(sizeof(SlotHdr) == 4096, "slot header must be 4 KiB");

struct Seg {
  std::string name;
  int fd = -1;
  uint8_t* base = nullptr;
  uint64_t total = 0;
  bool pinned = false;
  // background population (edl_shm_populate_async): pieces handed out by an atomic cursor
  std::vector<std::thread> pop;
  std::atomic<uint64_t> pop_next{0}, pop_done{0};
  std::atomic<bool> pop_stop{false};
  uint64_t pop_bytes = 0;
  bool pop_map = true;  // also map the populated pages into this process (see populate_async)
  SegHdr* hdr() { return reinterpret_cast<SegHdr*>(base); }
  SlotHdr* slot(int i) { return reinterpret_cast<SlotHdr*>(base + kHdr * (1 + i)); }
  uint8_t* data(int i) {
    return base + kHdr * (1 + hdr()->nslots) + (uint64_t)i * hdr()->slot_bytes;
  }
};

int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return (int64_t)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

uint64_t round_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// One read per 64 KiB: a read fault on a shared tmpfs mapping maps 16 pages at once
// (fault-around), writable.  The values are discarded, so a snapshot writing the same
// pages concurrently is harmless; ThreadSanitizer is told not to flag that.
__attribute__((no_sanitize("thread"))) void touch_pages(const uint8_t* p, uint64_t len) {
  volatile uint8_t sink = 0;
  for (uint64_t o = 0; o < len; o += 65536) sink = sink + p[o];
  (void)sink;
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// Persistent memcpy threads: run() splits one copy into one 64-byte-aligned stripe per
// thread and returns when every stripe is done.  Host DRAM <-> pinned staging copies of
// tens of GB need many cores: one thread moves ~6-10 GB/s out of shm pages.
class CopyPool {
 public:
  explicit CopyPool(int threads) : n_(threads < 1 ? 1 : threads) {
    for (int t = 0; t < n_; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_job_.notify_all();
    for (auto& t : th_) t.join();
  }
  // prefault: read one byte per 64 KiB of the destination stripe first.  On a fresh mapping
  // of existing tmpfs pages each such read fault maps 16 pages (the kernel's fault-around),
  // writable for a shared shmem mapping, so the copy then takes no fault at all instead of
  // one per 4 KiB page (2.7x the throughput of a plain copy into a fresh window, measured).
  void run(uint8_t* dst, const uint8_t* src, uint64_t n, bool prefault = false) {
    std::unique_lock<std::mutex> lk(mu_);
    dst_ = dst;
    src_ = src;
    len_ = n;
    prefault_ = prefault;
    pending_ = n_;
    ++gen_;
    cv_job_.notify_all();
    cv_done_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      uint8_t* dst;
      const uint8_t* src;
      uint64_t n;
      bool pf;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_job_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        dst = dst_;
        src = src_;
        n = len_;
        pf = prefault_;
      }
      const uint64_t per = ((n + n_ - 1) / n_ + 63) & ~uint64_t(63);
      const uint64_t lo = per * t;
      if (lo < n) {
        const uint64_t len = (lo + per > n) ? n - lo : per;
        if (pf) {
          volatile uint8_t sink = 0;
          for (uint64_t o = 0; o < len; o += 65536) sink = sink + dst[lo + o];
          (void)sink;
        }
        memcpy(dst + lo, src + lo, len);
      }
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) cv_done_.notify_one();
    }
  }
  const int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_job_, cv_done_;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  uint64_t len_ = 0;
  bool prefault_ = false;
};

}  // namespace

extern "C" {

// create=1: create (or resize) the segment; create=0: open an existing one.
void* edl_shm_open(const char* name, uint64_t slot_bytes, int nslots, int create) {
  if (!name) return nullptr;
  auto* s = new Seg();
  s->name = name;
  int flags = O_RDWR | (create ? O_CREAT : 0);
  s->fd = shm_open(name, flags, 0600);
  if (s->fd < 0) {
    delete s;
    return nullptr;
  }
  if (create) {
    if (nslots <= 0) nslots = 2;
    slot_bytes = round_up(slot_bytes ? slot_bytes : 4096, 2 << 20);
    s->total = kHdr * (1 + nslots) + slot_bytes * nslots;
    struct stat st;
    fstat(s->fd, &st);
    bool fresh = (uint64_t)st.st_size != s->total;
    if (fresh && ftruncate(s->fd, (off_t)s->total) != 0) {
      close(s->fd);
      delete s;
      return nullptr;
    }
    s->base = (uint8_t*)mmap(nullptr, s->total, PROT_READ | PROT_WRITE, MAP_SHARED, s->fd, 0);
    if (s->base == MAP_FAILED) {
      close(s->fd);
      delete s;
      return nullptr;
    }
    SegHdr* h = s->hdr();
    if (fresh || memcmp(h->magic, "EDLSHM01", 8) != 0 || h->slot_bytes != slot_bytes) {
      memset(s->base, 0, kHdr * (1 + nslots));
      memcpy(h->magic, "EDLSHM01", 8);
      h->version = 1;
      h->slot_bytes = slot_bytes;
      h->nslots = (uint32_t)nslots;
      h->current = -1;
      h->gen = 0;
    }
  } else {
    struct stat st;
    if (fstat(s->fd, &st) != 0 || (uint64_t)st.st_size < kHdr) {
      close(s->fd);
      delete s;
      return nullptr;
    }
    s->total = (uint64_t)st.st_size;
    s->base = (uint8_t*)mmap(nullptr, s->total, PROT_READ | PROT_WRITE, MAP_SHARED, s->fd, 0);
    if (s->base == MAP_FAILED || memcmp(s->hdr()->magic, "EDLSHM01", 8) != 0) {
      close(s->fd);
      delete s;
      return nullptr;
    }
  }
  return s;
}

// Page-lock every slot for DMA (idempotent).  Returns a hipError_t.
int edl_shm_pin(void* h) {
  auto* s = static_cast<Seg*>(h);
  if (s->pinned) return 0;
  uint8_t* d0 = s->data(0);
  uint64_t bytes = s->hdr()->slot_bytes * s->hdr()->nslots;
  hipError_t e = hipHostRegister(d0, bytes, hipHostRegisterPortable);
  if (e == hipSuccess) s->pinned = true;
  return (int)e;
}

// Populate this process's page tables for every slot (MADV_POPULATE_READ, in
// `threads` parallel ranges).  A hot standby does this ahead of any failure so
// the restore's staging memcpy never takes a page fault.  Returns 0 or -errno.
int edl_shm_prefault(void* h, int threads) {
  auto* s = static_cast<Seg*>(h);
#ifndef MADV_POPULATE_READ
#define MADV_POPULATE_READ 22
#endif
  uint8_t* d0 = s->data(0);
  const uint64_t bytes = s->hdr()->slot_bytes * s->hdr()->nslots;
  if (threads < 1) threads = 1;
  const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  const uint64_t per = round_up((bytes + threads - 1) / threads, page);
  std::atomic<int> err{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    const uint64_t lo = per * t;
    if (lo >= bytes) break;
    const uint64_t len = lo + per > bytes ? bytes - lo : per;
    ts.emplace_back([&, lo, len] {
      if (madvise(d0 + lo, len, MADV_POPULATE_READ) != 0) {
        // older kernels: touch one byte per page
        volatile uint8_t sink = 0;
        for (uint64_t o = 0; o < len; o += page) sink ^= d0[lo + o];
        (void)sink;
        err = errno;
      }
    });
  }
  for (auto& t : ts) t.join();
  return 0;
}

void* edl_shm_data(void* h, int slot) { return static_cast<Seg*>(h)->data(slot); }
uint64_t edl_shm_slot_bytes(void* h) { return static_cast<Seg*>(h)->hdr()->slot_bytes; }
int edl_shm_nslots(void* h) { return (int)static_cast<Seg*>(h)->hdr()->nslots; }
int edl_shm_current(void* h) { return __atomic_load_n(&static_cast<Seg*>(h)->hdr()->current, __ATOMIC_ACQUIRE); }

// Claim the slot to write next (never the current one) and mark it WRITING.
int edl_shm_begin(void* h) {
  auto* s = static_cast<Seg*>(h);
  int cur = edl_shm_current(h);
  int n = (int)s->hdr()->nslots;
  int slot = (cur + 1) % n;
  if (slot < 0) slot = 0;
  __atomic_store_n(&s->slot(slot)->state, kWriting, __ATOMIC_RELEASE);
  return slot;
}

int edl_shm_commit(void* h, int slot, int64_t step, int64_t epoch, uint64_t nbytes, uint64_t checksum,
                   const char* meta) {
  auto* s = static_cast<Seg*>(h);
  if (slot < 0 || slot >= (int)s->hdr()->nslots) return -EINVAL;
  if (nbytes > s->hdr()->slot_bytes) return -E2BIG;
  SlotHdr* sh = s->slot(slot);
  sh->step = step;
  sh->epoch = epoch;
  sh->nbytes = nbytes;
  sh->checksum = checksum;
  sh->ts_ns = now_ns();
  memset(sh->meta, 0, sizeof(sh->meta));
  if (meta) strncpy(sh->meta, meta, sizeof(sh->meta) - 1);
  sh->seq = s->hdr()->gen + 1;
  __atomic_store_n(&sh->state, kCommitted, __ATOMIC_RELEASE);
  __atomic_store_n(&s->hdr()->current, slot, __ATOMIC_RELEASE);
  __atomic_add_fetch(&s->hdr()->gen, 1, __ATOMIC_ACQ_REL);
  msync(s->base, kHdr * (1 + s->hdr()->nslots), MS_ASYNC);
  return 0;
}

// Latest committed slot (or -1) and its header fields.
int edl_shm_latest(void* h, int64_t* step, int64_t* epoch, uint64_t* nbytes, uint64_t* checksum, char* meta,
                   int metalen) {
  auto* s = static_cast<Seg*>(h);
  int cur = edl_shm_current(h);
  if (cur < 0) return -1;
  SlotHdr* sh = s->slot(cur);
  if (__atomic_load_n(&sh->state, __ATOMIC_ACQUIRE) != kCommitted) return -1;
  if (step) *step = sh->step;
  if (epoch) *epoch = sh->epoch;
  if (nbytes) *nbytes = sh->nbytes;
  if (checksum) *checksum = sh->checksum;
  if (meta && metalen > 0) {
    strncpy(meta, sh->meta, (size_t)metalen - 1);
    meta[metalen - 1] = 0;
  }
  return cur;
}

// Header of a specific slot: returns its state (0 empty, 1 writing, 2 committed).
int edl_shm_slot_info(void* h, int slot, int64_t* step, int64_t* epoch, uint64_t* nbytes, uint64_t* checksum,
                      char* meta, int metalen) {
  auto* s = static_cast<Seg*>(h);
  if (slot < 0 || slot >= (int)s->hdr()->nslots) return -EINVAL;
  SlotHdr* sh = s->slot(slot);
  int st = (int)__atomic_load_n(&sh->state, __ATOMIC_ACQUIRE);
  if (step) *step = sh->step;
  if (epoch) *epoch = sh->epoch;
  if (nbytes) *nbytes = sh->nbytes;
  if (checksum) *checksum = sh->checksum;
  if (meta && metalen > 0) {
    strncpy(meta, sh->meta, (size_t)metalen - 1);
    meta[metalen - 1] = 0;
  }
  return st;
}

// Populate every slot's pages in `threads` background threads (fallocate over 64 MiB pieces).
// First-touch of tmpfs pages runs at only ~4-5 GB/s however many threads fault them
// (measured on the MI355X box: a snapshot's copy into a never-written 96 GB slot stalled the step
// for 25 s), so a segment is populated off the training path as soon as it exists, and a
// snapshot waits for (or skips) an unfinished population instead of faulting inside its copy.
// Returns 0, or -1 if a population is already running.
int edl_shm_populate_async(void* h, int threads) {
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
  auto* s = static_cast<Seg*>(h);
  if (!s->pop.empty()) return -1;
  if (threads < 1) threads = 1;
  const uint64_t piece = 64ull << 20;
  s->pop_bytes = s->hdr()->slot_bytes * s->hdr()->nslots;
  s->pop_next = 0;
  s->pop_done = 0;
  uint8_t* d0 = s->data(0);
  for (int t = 0; t < threads; ++t) {
    s->pop.emplace_back([s, d0, piece] {
      for (;;) {
        if (s->pop_stop.load(std::memory_order_relaxed)) return;
        const uint64_t lo = s->pop_next.fetch_add(piece);
        if (lo >= s->pop_bytes) return;
        const uint64_t len = lo + piece > s->pop_bytes ? s->pop_bytes - lo : piece;
        // fallocate allocates the file's pages (the slow first touch, ~4 GB/s here); one read
        // per 64 KiB then maps them into this process 16 pages per fault (fault-around), so a
        // snapshot's copy takes no page fault.  Kernels / filesystems without fallocate: fault
        // the pages in directly.
        if (fallocate(s->fd, 0, (off_t)(d0 - s->base + lo), (off_t)len) != 0 &&
            madvise(d0 + lo, len, MADV_POPULATE_WRITE) != 0)
          madvise(d0 + lo, len, MADV_POPULATE_READ);
        if (s->pop_map) touch_pages(d0 + lo, len);
        s->pop_done.fetch_add(len);
      }
    });
  }
  return 0;
}

// Bytes populated so far and the total (0 / 0: no population started).
uint64_t edl_shm_populate_progress(void* h, uint64_t* total) {
  auto* s = static_cast<Seg*>(h);
  if (total) *total = s->pop.empty() ? 0 : s->pop_bytes;
  return s->pop.empty() ? 0 : s->pop_done.load();
}

static void populate_join(Seg* s) {
  s->pop_stop = true;
  for (auto& t : s->pop) t.join();
  s->pop.clear();
}

int edl_shm_close(void* h, int unlink_seg) {
  auto* s = static_cast<Seg*>(h);
  if (!s) return 0;
  populate_join(s);
  if (s->pinned) hipHostUnregister(s->data(0));
  munmap(s->base, s->total);
  close(s->fd);
  if (unlink_seg) shm_unlink(s->name.c_str());
  delete s;
  return 0;
}

int edl_shm_unlink(const char* name) { return shm_unlink(name) == 0 ? 0 : -errno; }

// the segment's file descriptor (identity checks: does a /dev/shm name still refer to it?)
int edl_shm_fd(void* h) { return h ? static_cast<Seg*>(h)->fd : -1; }

// Re-use an already mapped (and page-locked) segment for another shard layout
// after a world change: invalidate both slots FIRST (no reader may take the old
// layout's bytes for the new name), then atomically rename the /dev/shm file
// (replacing a stale one of that name).  Mappings stay valid across the rename,
// so the multi-GB hipHostRegister is not repeated.  Returns 0 or -errno.
int edl_shm_reassign(void* h, const char* new_name) {
  auto* s = static_cast<Seg*>(h);
  if (!s || !new_name || new_name[0] != '/') return -EINVAL;
  for (uint32_t i = 0; i < s->hdr()->nslots; ++i) __atomic_store_n(&s->slot(i)->state, kEmpty, __ATOMIC_RELEASE);
  __atomic_store_n(&s->hdr()->current, -1, __ATOMIC_RELEASE);
  msync(s->base, kHdr * (1 + s->hdr()->nslots), MS_SYNC);
  const std::string from = "/dev/shm" + s->name, to = std::string("/dev/shm") + new_name;
  if (from != to && rename(from.c_str(), to.c_str()) != 0) return -errno;
  s->name = new_name;
  return 0;
}

// Re-use the segment for a new layout WITHOUT dropping the newest snapshot of the
// old one: every slot except the current one is invalidated and the file gets a
// second name (hard link) for the new layout.  Until the caller unlinks the old
// name (once this rank's first new-layout snapshot has committed, just before the
// kept slot is overwritten), a whole-job restart still finds the old world's
// complete snapshot set.  Slots carry their layout in `meta`, so readers of either
// name tell old-layout and new-layout slots apart.  Returns 0 or -errno.
int edl_shm_relink(void* h, const char* new_name) {
  auto* s = static_cast<Seg*>(h);
  if (!s || !new_name || new_name[0] != '/') return -EINVAL;
  const int32_t cur = __atomic_load_n(&s->hdr()->current, __ATOMIC_ACQUIRE);
  for (uint32_t i = 0; i < s->hdr()->nslots; ++i)
    if ((int32_t)i != cur) __atomic_store_n(&s->slot(i)->state, kEmpty, __ATOMIC_RELEASE);
  msync(s->base, kHdr * (1 + s->hdr()->nslots), MS_SYNC);
  const std::string from = "/dev/shm" + s->name, to = std::string("/dev/shm") + new_name;
  if (from != to) {
    unlink(to.c_str());  // a stale segment of that name (an older run's layout)
    if (link(from.c_str(), to.c_str()) != 0) return -errno;
  }
  s->name = new_name;
  return 0;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// asynchronous snapshot engine
// ---------------------------------------------------------------------------
namespace {

struct Job {
  int64_t ticket;
  Seg* seg;
  int slot;
  int64_t step, epoch;
  uint64_t nbytes;
  int64_t checksum_off;
  std::string meta;
  hipEvent_t done;
  // staged form (slot not page-locked): the worker thread copies through pinned stages
  bool staged = false;
  hipEvent_t ready = nullptr;
  std::vector<uint64_t> ptrs, sizes, offs;
};

struct Engine {
  int device = 0;
  hipStream_t side = nullptr;
  std::thread committer;
  std::mutex mu;
  std::condition_variable cv;
  std::condition_variable cv_reads;      // staged jobs: device reads finished
  std::deque<Job> queue;
  std::map<int64_t, int> status;         // 0 pending, 1 committed, <0 error
  std::map<int64_t, hipEvent_t> events;  // completion events (for fences)
  std::map<int64_t, bool> reads;         // staged tickets: true once every D2H has landed
  int64_t next = 1;
  bool stop = false;
  uint64_t chunk = 256ull << 20;
  // staged snapshots: pinned staging ring + memcpy pool, created at the first staged job
  uint64_t stage_bytes = 128ull << 20;
  int nstage = 4;
  int threads = 16;
  std::vector<void*> stage;
  std::vector<hipEvent_t> sev;
  CopyPool* pool = nullptr;
  bool windowed = false;                 // EDL_SNAPSHOT_WINDOW=1: copy through per-piece windows
  double last_staged[4] = {0, 0, 0, 0};  // d2h_wait_s, copy_s, total_s, bytes of the last staged job
};

// Device buffers -> (pageable) slot through the pinned staging ring: D2H of chunk c into
// stage c % S on the (CU-masked) side stream while the pool copies an earlier stage out to
// the shm pages.  Marks the ticket's device reads done as soon as the last D2H has landed
// (fences wait for that, not for the host copies), then returns after the last host copy.
hipError_t run_staged(Engine* e, Job& j) {
  hipError_t err = hipSuccess;
  if (!e->pool) {
    e->stage.assign(e->nstage, nullptr);
    e->sev.assign(e->nstage, nullptr);
    for (int i = 0; i < e->nstage && err == hipSuccess; ++i) {
      err = hipHostMalloc(&e->stage[i], e->stage_bytes, hipHostMallocDefault);
      if (err == hipSuccess) err = hipEventCreateWithFlags(&e->sev[i], hipEventDisableTiming);
    }
    if (err != hipSuccess) return err;
    e->pool = new CopyPool(e->threads);
  }
  struct Piece {
    const uint8_t* src;
    uint64_t fo;  // byte offset in the segment file
    uint64_t n;
  };
  std::vector<Piece> pieces;
  const uint64_t slot_fo = (uint64_t)(j.seg->data(j.slot) - j.seg->base);
  for (size_t b = 0; b < j.ptrs.size(); ++b)
    for (uint64_t off = 0; off < j.sizes[b]; off += e->stage_bytes)
      pieces.push_back({(const uint8_t*)j.ptrs[b] + off, slot_fo + j.offs[b] + off,
                        j.sizes[b] - off < e->stage_bytes ? j.sizes[b] - off : e->stage_bytes});
  static const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE);
  const double t_start = now_s();
  double wait_s = 0, copy_s = 0;
  uint64_t bytes = 0;
  const size_t S = (size_t)e->nstage, P = pieces.size();
  err = hipStreamWaitEvent(e->side, j.ready, 0);
  auto drain = [&](size_t c) {  // stage c % S holds piece c: wait for its D2H, copy it out
    const int k = (int)(c % S);
    double t0 = now_s();
    hipError_t r = hipEventSynchronize(e->sev[k]);
    wait_s += now_s() - t0;
    if (r != hipSuccess) return r;
    if (c + 1 == P) {  // every device read has landed: release the fence before the host copy
      std::lock_guard<std::mutex> g(e->mu);
      e->reads[j.ticket] = true;
      e->cv_reads.notify_all();
    }
    t0 = now_s();
    // Written through a window mapped for this piece only, not through the segment's
    // process-wide mapping: every page of a snapshot slot mapped in this process is a page
    // table entry the kernel must tear down when the process dies, and the operator hands
    // the GPU to a replacement only after that (19 ms per GB on the MI355X box,
    // scripts/exit_cost_probe.cpp: ~3.6 s for a 192 GB slot pair).  The window costs a
    // minor fault per page and a 128 MB unmap per piece, off the training thread.
    const uint64_t a = pieces[c].fo & ~(page - 1), d = pieces[c].fo - a, len = d + pieces[c].n;
    uint8_t* w = e->windowed ? (uint8_t*)mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, j.seg->fd, (off_t)a)
                             : (uint8_t*)MAP_FAILED;
    if (w != (uint8_t*)MAP_FAILED) {
      e->pool->run(w + d, (const uint8_t*)e->stage[k], pieces[c].n, true);
      munmap(w, len);
    } else {
      e->pool->run(j.seg->base + pieces[c].fo, (const uint8_t*)e->stage[k], pieces[c].n, true);
    }
    copy_s += now_s() - t0;
    bytes += pieces[c].n;
    return hipSuccess;
  };
  for (size_t c = 0; c < P && err == hipSuccess; ++c) {
    const int k = (int)(c % S);
    if (c >= S) err = drain(c - S);
    if (err == hipSuccess) err = hipMemcpyAsync(e->stage[k], pieces[c].src, pieces[c].n, hipMemcpyDeviceToHost,
                                                e->side);
    if (err == hipSuccess) err = hipEventRecord(e->sev[k], e->side);
  }
  for (size_t c = P > S ? P - S : 0; c < P && err == hipSuccess; ++c) err = drain(c);
  if (P == 0 && err == hipSuccess) err = hipStreamSynchronize(e->side);
  std::lock_guard<std::mutex> g(e->mu);
  e->last_staged[0] = wait_s;
  e->last_staged[1] = copy_s;
  e->last_staged[2] = now_s() - t_start;
  e->last_staged[3] = (double)bytes;
  return err;
}

void commit_loop(Engine* e) {
  hipSetDevice(e->device);
  for (;;) {
    Job j;
    {
      std::unique_lock<std::mutex> g(e->mu);
      e->cv.wait(g, [&] { return e->stop || !e->queue.empty(); });
      if (e->queue.empty()) return;
      j = e->queue.front();
      e->queue.pop_front();
    }
    hipError_t err = j.staged ? run_staged(e, j) : hipEventSynchronize(j.done);
    if (j.ready) hipEventDestroy(j.ready);
    int st = 1;
    if (err != hipSuccess) {
      st = -(int)err;
    } else {
      uint64_t cs = 0;
      if (j.checksum_off >= 0) memcpy(&cs, j.seg->data(j.slot) + j.checksum_off, sizeof(cs));
      if (edl_shm_commit(j.seg, j.slot, j.step, j.epoch, j.nbytes, cs, j.meta.c_str()) != 0) st = -1;
    }
    std::lock_guard<std::mutex> g(e->mu);
    e->status[j.ticket] = st;
    if (j.staged) {
      e->reads[j.ticket] = true;  // also on failure: a fence never waits forever
      e->cv_reads.notify_all();
    }
  }
}

}  // namespace

extern "C" {

// copy_cus > 0: the side stream is restricted to that many CUs, spread over the
// 8 XCDs.  On MI355X / ROCm 7 a D2H hipMemcpyAsync into page-locked memory runs
// as a blit KERNEL (__amd_rocclr_copyBuffer), not on an SDMA engine, so an
// unrestricted copy competes with training kernels for every CU: measured
// (scripts/d2h_overlap_probe.py) GEMMs lose 9 % while a snapshot streams on an
// unmasked stream vs 2.7 % with 8 CUs, and the copy itself gets faster
// (48.5 -> 51.8 GB/s).  A CU-masked stream is a blocking stream: callers must
// not run compute on the legacy NULL stream (the trainer uses a pool stream).
void* edl_ckpt_engine_create(int device, uint64_t chunk_bytes, int copy_cus) {
  auto* e = new Engine();
  e->device = device;
  const char* win = getenv("EDL_SNAPSHOT_WINDOW");
  e->windowed = win && win[0] == '1';
  if (chunk_bytes) e->chunk = chunk_bytes;
  if (hipSetDevice(device) != hipSuccess) {
    delete e;
    return nullptr;
  }
  hipError_t err = hipErrorUnknown;
  if (copy_cus > 0) {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
    if (ncu >= 8 && copy_cus < ncu) {
      // a rank under a Brain CU plan (EDL_CU_MASK, hex over the CUs) copies on CUs of its
      // own share only: the engine's CUs are picked from the plan's set
      std::vector<uint32_t> allowed((ncu + 31) / 32, 0xFFFFFFFFu);
      if (const char* plan = getenv("EDL_CU_MASK")) {
        std::fill(allowed.begin(), allowed.end(), 0u);
        const char* p = plan;
        if (p[0] == '0' && (p[1] == 'x' || p[1] == 'X')) p += 2;
        const int len = (int)strlen(p);
        for (int i = 0; i < len; ++i) {  // hex digit i from the right holds CUs 4i .. 4i+3
          const char ch = p[len - 1 - i];
          const int v = (ch >= '0' && ch <= '9') ? ch - '0' : (ch >= 'a' && ch <= 'f') ? ch - 'a' + 10
                        : (ch >= 'A' && ch <= 'F') ? ch - 'A' + 10 : 0;
          for (int b = 0; b < 4; ++b)
            if ((v >> b) & 1 && 4 * i + b < ncu) allowed[(4 * i + b) / 32] |= 1u << ((4 * i + b) % 32);
        }
      }
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      const int per_xcd = ncu / 8;
      int picked = 0;
      for (int i = 0; i < ncu && picked < copy_cus; ++i) {
        const int xcd = i % 8, c = (i / 8) % per_xcd;
        const int cu = c * 8 + xcd;  // hardware CU ids interleave the XCDs
        if (!((allowed[cu / 32] >> (cu % 32)) & 1u)) continue;
        mask[cu / 32] |= 1u << (cu % 32);
        ++picked;
      }
      if (picked > 0) err = hipExtStreamCreateWithCUMask(&e->side, (uint32_t)mask.size(), mask.data());
    }
  }
  if (err != hipSuccess) {
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);  // lo = least priority
    err = hipStreamCreateWithPriority(&e->side, hipStreamNonBlocking, lo);
  }
  if (err != hipSuccess) {
    delete e;
    return nullptr;
  }
  e->committer = std::thread(commit_loop, e);
  return e;
}

// Enqueue a snapshot of nbuf device buffers into the free slot of `seg`.
// dev_ptrs/sizes/offsets: per buffer source pointer, byte size, byte offset in
// the slot.  after_stream: the compute stream whose current position marks the
// consistent state.  checksum_off: slot offset of an 8-byte checksum that is
// part of the copied buffers (published in the header), or -1.
// Returns a ticket (>0) or a negative hipError_t.
int64_t edl_ckpt_snapshot(void* eng, void* seg, int nbuf, const uint64_t* dev_ptrs, const uint64_t* sizes,
                          const uint64_t* offsets, hipStream_t after_stream, int64_t step, int64_t epoch,
                          int64_t checksum_off, const char* meta) {
  auto* e = static_cast<Engine*>(eng);
  auto* s = static_cast<Seg*>(seg);
  hipSetDevice(e->device);
  uint64_t total = 0;
  for (int i = 0; i < nbuf; ++i) {
    if (offsets[i] + sizes[i] > s->hdr()->slot_bytes) return -(int64_t)hipErrorInvalidValue;
    if (offsets[i] + sizes[i] > total) total = offsets[i] + sizes[i];
  }
  int slot = edl_shm_begin(s);
  if (!s->pinned) {
    // pageable slot: the worker thread streams it through the pinned staging ring
    Job j{0, s, slot, step, epoch, total, checksum_off, meta ? meta : "", nullptr};
    j.staged = true;
    hipError_t err = hipEventCreateWithFlags(&j.ready, hipEventDisableTiming);
    if (err == hipSuccess) err = hipEventRecord(j.ready, after_stream);
    if (err != hipSuccess) {
      if (j.ready) hipEventDestroy(j.ready);
      return -(int64_t)err;
    }
    j.ptrs.assign(dev_ptrs, dev_ptrs + nbuf);
    j.sizes.assign(sizes, sizes + nbuf);
    j.offs.assign(offsets, offsets + nbuf);
    std::lock_guard<std::mutex> g(e->mu);
    j.ticket = e->next++;
    e->status[j.ticket] = 0;
    e->reads[j.ticket] = false;
    e->queue.push_back(std::move(j));
    e->cv.notify_one();
    return e->next - 1;
  }
  hipEvent_t ready, done;
  hipEventCreateWithFlags(&ready, hipEventDisableTiming);
  hipEventCreateWithFlags(&done, hipEventDisableTiming);
  hipError_t err = hipEventRecord(ready, after_stream);
  if (err == hipSuccess) err = hipStreamWaitEvent(e->side, ready, 0);
  uint8_t* dst = s->data(slot);
  for (int i = 0; i < nbuf && err == hipSuccess; ++i) {
    for (uint64_t off = 0; off < sizes[i] && err == hipSuccess; off += e->chunk) {
      uint64_t n = sizes[i] - off < e->chunk ? sizes[i] - off : e->chunk;
      err = hipMemcpyAsync(dst + offsets[i] + off, (const uint8_t*)dev_ptrs[i] + off, n, hipMemcpyDeviceToHost,
                           e->side);
    }
  }
  if (err == hipSuccess) err = hipEventRecord(done, e->side);
  hipEventDestroy(ready);
  if (err != hipSuccess) {
    hipEventDestroy(done);
    return -(int64_t)err;
  }
  std::lock_guard<std::mutex> g(e->mu);
  int64_t t = e->next++;
  e->status[t] = 0;
  e->events[t] = done;
  e->queue.push_back(Job{t, s, slot, step, epoch, total, checksum_off, meta ? meta : "", done});
  e->cv.notify_one();
  return t;
}

// Make `stream` wait until snapshot `ticket` has finished reading device memory.
int edl_ckpt_fence(void* eng, int64_t ticket, hipStream_t stream) {
  auto* e = static_cast<Engine*>(eng);
  hipEvent_t ev = nullptr;
  {
    std::unique_lock<std::mutex> g(e->mu);
    auto rd = e->reads.find(ticket);
    if (rd != e->reads.end()) {
      // staged snapshot: its D2H copies are issued by the worker thread as stages free up,
      // so there is no event to chain the stream on; wait on the host for the last one
      e->cv_reads.wait(g, [&] { return rd->second; });
      return 0;
    }
    auto it = e->events.find(ticket);
    if (it == e->events.end()) return 0;
    ev = it->second;
  }
  return (int)hipStreamWaitEvent(stream, ev, 0);
}

// 0 pending, 1 committed, negative = error.  Committed tickets release their event.
int edl_ckpt_status(void* eng, int64_t ticket) {
  auto* e = static_cast<Engine*>(eng);
  std::lock_guard<std::mutex> g(e->mu);
  auto it = e->status.find(ticket);
  if (it == e->status.end()) return 1;
  int st = it->second;
  if (st != 0) {
    auto ev = e->events.find(ticket);
    if (ev != e->events.end()) {
      hipEventDestroy(ev->second);
      e->events.erase(ev);
    }
    e->reads.erase(ticket);
    e->status.erase(it);
  }
  return st;
}

int edl_ckpt_wait(void* eng, int64_t ticket, int timeout_ms) {
  for (int waited = 0;; waited += 1) {
    int st = edl_ckpt_status(eng, ticket);
    if (st != 0) return st;
    if (timeout_ms >= 0 && waited >= timeout_ms) return 0;
    usleep(1000);
  }
}

// Host slot -> device buffers (H2D on `stream`).
int edl_ckpt_restore(void* seg, int slot, int nbuf, const uint64_t* dev_ptrs, const uint64_t* sizes,
                     const uint64_t* offsets, hipStream_t stream) {
  auto* s = static_cast<Seg*>(seg);
  if (slot < 0) slot = edl_shm_current(s);
  if (slot < 0) return -1;
  const uint8_t* src = s->data(slot);
  for (int i = 0; i < nbuf; ++i) {
    hipError_t err = hipMemcpyAsync((void*)dev_ptrs[i], src + offsets[i], sizes[i], hipMemcpyHostToDevice, stream);
    if (err != hipSuccess) return (int)err;
  }
  return 0;
}

// Fast restore from (pageable) shm: multi-threaded memcpy into two pinned
// staging buffers, each drained by an async H2D copy on `stream`; the CPU copy
// of chunk i+1 overlaps the DMA of chunk i.  Blocks until done.
int edl_ckpt_restore_pipelined(void* seg, int slot, int nbuf, const uint64_t* dev_ptrs, const uint64_t* sizes,
                               const uint64_t* offsets, hipStream_t stream, uint64_t chunk, int threads) {
  auto* s = static_cast<Seg*>(seg);
  if (slot < 0) slot = edl_shm_current(s);
  if (slot < 0) return -1;
  if (chunk == 0) chunk = 256ull << 20;
  if (threads <= 0) threads = 8;
  void* stage[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  hipError_t err = hipSuccess;
  for (int i = 0; i < 2 && err == hipSuccess; ++i) {
    err = hipHostMalloc(&stage[i], chunk, hipHostMallocDefault);
    if (err == hipSuccess) err = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
  }
  bool used[2] = {false, false};
  int k = 0;
  const uint8_t* base = s->data(slot);
  for (int b = 0; b < nbuf && err == hipSuccess; ++b) {
    for (uint64_t off = 0; off < sizes[b] && err == hipSuccess; off += chunk, k ^= 1) {
      const uint64_t n = sizes[b] - off < chunk ? sizes[b] - off : chunk;
      if (used[k]) err = hipEventSynchronize(ev[k]);  // staging buffer k free again
      if (err != hipSuccess) break;
      const uint8_t* src = base + offsets[b] + off;
      uint8_t* dst = (uint8_t*)stage[k];
      const uint64_t per = (n + threads - 1) / threads;
      std::vector<std::thread> ts;
      for (int t = 0; t < threads; ++t) {
        const uint64_t lo = per * t;
        if (lo >= n) break;
        const uint64_t len = (lo + per > n) ? n - lo : per;
        ts.emplace_back([=] { memcpy(dst + lo, src + lo, len); });
      }
      for (auto& th : ts) th.join();
      err = hipMemcpyAsync((uint8_t*)dev_ptrs[b] + off, dst, n, hipMemcpyHostToDevice, stream);
      if (err == hipSuccess) err = hipEventRecord(ev[k], stream);
      used[k] = true;
    }
  }
  if (err == hipSuccess) err = hipStreamSynchronize(stream);
  for (int i = 0; i < 2; ++i) {
    if (ev[i]) hipEventDestroy(ev[i]);
    if (stage[i]) hipHostFree(stage[i]);
  }
  return (int)err;
}

// Restore, v2: a persistent pool of `threads` copy threads (one stripe of every chunk each)
// and `stages` pinned staging buffers; chunk c is copied into stage c % stages while the DMA
// of the previous chunks drains.  stats (may be null) receives {copy_s, dma_wait_s, total_s,
// bytes}: where the time goes (host memcpy out of the shm pages vs waiting for the H2D
// engine), so the restore can be tuned from a measurement.  Blocks until done.
int edl_ckpt_restore_pipelined2(void* seg, int slot, int nbuf, const uint64_t* dev_ptrs, const uint64_t* sizes,
                                const uint64_t* offsets, hipStream_t stream, uint64_t chunk, int threads, int stages,
                                double* stats) {
  auto* s = static_cast<Seg*>(seg);
  if (slot < 0) slot = edl_shm_current(s);
  if (slot < 0) return -1;
  if (chunk == 0) chunk = 128ull << 20;
  if (threads <= 0) threads = 16;
  if (stages < 2) stages = 2;
  if (stages > 8) stages = 8;
  const double t_start = now_s();
  std::vector<void*> stage(stages, nullptr);
  std::vector<hipEvent_t> ev(stages, nullptr);
  std::vector<bool> used(stages, false);
  hipError_t err = hipSuccess;
  for (int i = 0; i < stages && err == hipSuccess; ++i) {
    err = hipHostMalloc(&stage[i], chunk, hipHostMallocDefault);
    if (err == hipSuccess) err = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
  }
  // the work list: (src, dst device pointer, bytes) per chunk
  struct Piece {
    const uint8_t* src;
    uint8_t* dst;
    uint64_t n;
  };
  std::vector<Piece> pieces;
  const uint8_t* base = s->data(slot);
  for (int b = 0; b < nbuf; ++b)
    for (uint64_t off = 0; off < sizes[b]; off += chunk)
      pieces.push_back({base + offsets[b] + off, (uint8_t*)dev_ptrs[b] + off,
                        sizes[b] - off < chunk ? sizes[b] - off : chunk});
  CopyPool pool(threads);
  double copy_s = 0.0, wait_s = 0.0;
  uint64_t bytes = 0;
  for (size_t c = 0; c < pieces.size() && err == hipSuccess; ++c) {
    const int k = (int)(c % stages);
    if (used[k]) {
      const double t0 = now_s();
      err = hipEventSynchronize(ev[k]);  // staging buffer k free again
      wait_s += now_s() - t0;
      if (err != hipSuccess) break;
    }
    const double t0 = now_s();
    pool.run((uint8_t*)stage[k], pieces[c].src, pieces[c].n);
    copy_s += now_s() - t0;
    err = hipMemcpyAsync(pieces[c].dst, stage[k], pieces[c].n, hipMemcpyHostToDevice, stream);
    if (err == hipSuccess) err = hipEventRecord(ev[k], stream);
    used[k] = true;
    bytes += pieces[c].n;
  }
  const double t0 = now_s();
  if (err == hipSuccess) err = hipStreamSynchronize(stream);
  wait_s += now_s() - t0;
  for (int i = 0; i < stages; ++i) {
    if (ev[i]) hipEventDestroy(ev[i]);
    if (stage[i]) hipHostFree(stage[i]);
  }
  if (stats) {
    stats[0] = copy_s;
    stats[1] = wait_s;
    stats[2] = now_s() - t_start;
    stats[3] = (double)bytes;
  }
  return (int)err;
}

// ---------------------------------------------------------------------------
// Step marks: one 4 KiB shm page per worker slot that survives the worker.  The worker's GPU
// writes, in stream order, the step whose optimizer update is about to start (begin) and the
// step whose update has finished (done) -- kernel-side system-scope stores (edl_ps_signal)
// into the page, page-locked and mapped for the device.  A replacement that adopted the dead
// worker's HBM (utils/vram.py) reads them: begin == done == K means the HBM holds exactly the
// state after step K (no update was in flight), so no snapshot needs restoring.
// ---------------------------------------------------------------------------
struct MarkPage {
  std::string name;
  int fd = -1;
  uint8_t* base = nullptr;
  bool pinned = false;
};

// Returns a handle; *host = the page, *dev = its device address (null unless pinned).
void* edl_mark_open(const char* name, int create, int pin, void** host, void** dev) {
  auto* m = new MarkPage();
  m->name = name;
  m->fd = shm_open(name, O_RDWR | (create ? O_CREAT : 0), 0600);
  if (m->fd < 0 || (create && ftruncate(m->fd, 4096) != 0)) {
    if (m->fd >= 0) close(m->fd);
    delete m;
    return nullptr;
  }
  m->base = (uint8_t*)mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, m->fd, 0);
  if (m->base == MAP_FAILED) {
    close(m->fd);
    delete m;
    return nullptr;
  }
  if (host) *host = m->base;
  if (dev) *dev = nullptr;
  if (pin && hipHostRegister(m->base, 4096, hipHostRegisterMapped) == hipSuccess) {
    m->pinned = true;
    void* d = nullptr;
    if (dev && hipHostGetDevicePointer(&d, m->base, 0) == hipSuccess) *dev = d;
  }
  return m;
}

void edl_mark_close(void* h, int unlink_page) {
  auto* m = static_cast<MarkPage*>(h);
  if (!m) return;
  if (m->pinned) hipHostUnregister(m->base);
  munmap(m->base, 4096);
  close(m->fd);
  if (unlink_page) shm_unlink(m->name.c_str());
  delete m;
}

// Staged-snapshot parameters (before the first staged job): stage size, ring depth, copy threads.
int edl_ckpt_engine_staging(void* eng, uint64_t stage_bytes, int nstage, int threads) {
  auto* e = static_cast<Engine*>(eng);
  std::lock_guard<std::mutex> g(e->mu);
  if (e->pool) return -1;
  if (stage_bytes) e->stage_bytes = round_up(stage_bytes, 2 << 20);
  if (nstage >= 2) e->nstage = nstage > 16 ? 16 : nstage;
  if (threads >= 1) e->threads = threads > 64 ? 64 : threads;
  return 0;
}

// {d2h_wait_s, copy_s, total_s, bytes} of the last finished staged snapshot.
void edl_ckpt_engine_staged_stats(void* eng, double* out) {
  auto* e = static_cast<Engine*>(eng);
  std::lock_guard<std::mutex> g(e->mu);
  for (int i = 0; i < 4; ++i) out[i] = e->last_staged[i];
}

int edl_shm_pinned(void* h) { return h && static_cast<Seg*>(h)->pinned ? 1 : 0; }

void edl_ckpt_engine_destroy(void* eng) {
  auto* e = static_cast<Engine*>(eng);
  if (!e) return;
  {
    std::lock_guard<std::mutex> g(e->mu);
    e->stop = true;
  }
  e->cv.notify_all();
  if (e->committer.joinable()) e->committer.join();
  for (auto& kv : e->events) hipEventDestroy(kv.second);
  delete e->pool;
  for (auto ev : e->sev)
    if (ev) hipEventDestroy(ev);
  for (auto p : e->stage)
    if (p) hipHostFree(p);
  if (e->side) hipStreamDestroy(e->side);
  delete e;
}

}  // extern "C"

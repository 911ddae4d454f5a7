// worker.cpp — native GPU worker API (see worker.h).
#include "worker.h"

#include <stdexcept>

namespace ss {

namespace {
template <typename T>
T* dev_alloc(size_t count) {
  void* p = nullptr;
  check_hip(hipMalloc(&p, count * sizeof(T) + 8), "GpuWorker: hipMalloc");
  return static_cast<T*>(p);
}
unsigned long long next_pow2(unsigned long long x) {
  unsigned long long p = 1;
  while (p < x) p <<= 1;
  return p;
}
SegList device_count_segs(const unsigned long long* count) {
  SegList sl{};
  sl.nseg = 1;
  sl.dev_count = reinterpret_cast<const long long*>(count);
  return sl;
}
}  // namespace

Handle::Handle(hipStream_t st) {
  hipEvent_t e;
  check_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "Handle: hipEventCreate");
  check_hip(hipEventRecord(e, st), "Handle: hipEventRecord");
  ev_ = std::shared_ptr<void>(e, [](void* p) { (void)hipEventDestroy((hipEvent_t)p); });
}

bool Handle::done() const {
  if (!ev_) return true;
  const hipError_t r = hipEventQuery((hipEvent_t)ev_.get());
  if (r == hipErrorNotReady) return false;
  check_hip(r, "Handle: hipEventQuery");
  return true;
}

void Handle::wait() const {
  if (ev_) check_hip(hipEventSynchronize((hipEvent_t)ev_.get()), "Handle: hipEventSynchronize");
}

GpuWorker::GpuWorker(const DevTable& t, unsigned long long* size_ctr, int* err,
                     const InitParams& init, const OptParams& opt, int G, long long max_keys)
    : t_(t), size_ctr_(size_ctr), err_(err), init_(init), opt_(opt), G_(G), max_keys_(max_keys) {
  if (max_keys < 1) throw std::invalid_argument("GpuWorker: max_keys must be >= 1");
  if (!size_ctr || !err) throw std::invalid_argument("GpuWorker: size counter / error word");
  const size_t m = (size_t)max_keys;
  scap_ = next_pow2(m + m / 2 + 1);  // dedup table load <= 2/3 with every key unique
  skeys_ = dev_alloc<uint64_t>(scap_);
  stag_ = dev_alloc<uint32_t>(scap_);
  slot_of_ = dev_alloc<uint32_t>(m);
  blk_cnt_ = dev_alloc<uint32_t>((size_t)dedup_cnt_words((long long)m, 1));
  frag_map_ = dev_alloc<int>(1);
  check_hip(hipMemset(frag_map_, 0, sizeof(int)), "GpuWorker: frag map");
  // the dedup's finish kernel returns the slots it claimed to EMPTY, so one
  // fill here keeps the scratch clean across calls
  check_hip(hipMemset(skeys_, 0xFF, scap_ * sizeof(uint64_t)), "GpuWorker: scratch fill");
  inv_ = dev_alloc<uint32_t>(m);
  ukeys_ = dev_alloc<uint64_t>(m);
  ucount_ = dev_alloc<unsigned long long>(1);
  slots_ = dev_alloc<long long>(m);
  urows_ = dev_alloc<float>(m * t_.dim);
}

GpuWorker::~GpuWorker() {
  for (void* p : {(void*)skeys_, (void*)stag_, (void*)slot_of_, (void*)blk_cnt_, (void*)frag_map_,
                  (void*)inv_, (void*)ukeys_, (void*)ucount_, (void*)slots_, (void*)urows_})
    if (p) (void)hipFree(p);
}

void GpuWorker::dedup(const uint64_t* keys, long long n, hipStream_t st) {
  if (n < 0 || n > max_keys_) throw std::invalid_argument("GpuWorker: n outside [0, max_keys]");
  RouteSpec rs{};
  rs.frag_map = frag_map_;
  rs.frag_num = 1;
  rs.nranks = 1;
  // push: the dedup zeroes the unique gradient rows it hands out (urows_)
  launch_dedup_route(keys, n, skeys_, stag_, scap_, slot_of_, rs, max_keys_, ucount_, ukeys_,
                     urows_, (int)t_.dim, blk_cnt_, inv_, st);
}

Handle GpuWorker::pull(const uint64_t* keys, long long n, float* vals, hipStream_t st) {
  dedup(keys, n, st);
  if (n > 0) {
    const SegList sl = device_count_segs(ucount_);
    launch_pull_unique(t_, ukeys_, sl, n, slots_, urows_, init_, size_ctr_, err_, G_, st);
    launch_gather_rows(urows_, inv_, n, (int)t_.dim, vals, st);
  }
  return Handle(st);
}

Handle GpuWorker::push(const uint64_t* keys, long long n, const float* grads, hipStream_t st) {
  dedup(keys, n, st);
  if (n > 0) {
    const SegList sl = device_count_segs(ucount_);
    launch_scatter_add_rows(grads, inv_, n, (int)t_.dim, urows_, st);
    launch_probe(t_, ukeys_, sl, n, slots_, init_, 1, size_ctr_, err_, G_, st);
    launch_apply(t_, slots_, urows_, sl, n, opt_, G_, st);
  }
  return Handle(st);
}

}  // namespace ss

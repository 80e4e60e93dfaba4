// runtime.hip — variant switches, per-device CU counts, last-launch record (runtime.hpp).
#include "runtime.hpp"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "specenh.h"

namespace specenh {
int set_error(int code, const std::string& msg);  // stft_psd.hip

namespace {

struct VariantName {
  const char* name;
  int dflt;
};
constexpr VariantName kVariants[V_COUNT] = {
    {"CONVT_PAIR", 0},      {"PATCH_NO_WL", 0},      {"PATCH_NO_K5", 0},
    {"PATCH_WSPLIT", -1},   {"CONV_NO_S2", 0},       {"CONV_NO_PATCH", 0},
    {"CONV_NO_C1MFMA", 0},  {"CONV_NO_NARROW", 0},   {"WGRAD_GENERIC", 0},
    {"WGRAD_NO_CO1", 0},    {"WGRAD_PERPHASE", 0},   {"SVD_GRAM_TILES", 0},
    {"TAIL_TILES", 0},      {"DECODER_UNFUSED", 0},  {"SVD_NO_TOP1", 0},
    {"CONV_NO_ROWS", 0},    {"CONVT_NO_ROWS", 0},    {"CONV1_NO_ROWS", 0},
    {"ENCODER_UNFUSED", 0},  {"STFT_NO_HOLD", 0},    {"D3_MAP", 0},
    {"ENC2_WPE2", 0},        {"CONVT_SHARED_RING", 0}, {"SVD_RECON_VALU", 0},
    {"ROWS_SHORT_LEAD", 0},  {"SVD_GRAM_F32", 0},
    {"SVD_RECON_BLOCKS", 0}, {"CONVT_PG", 0}, {"SVD_GZ_ROWS", 0}, {"EIG_SPLIT", 0}, {"CO1_VALU", 0},
    {"C1_MASK_MFMA", 1}, {"S2_MIN_NT", 2}, {"PATCH_MIN_WG", 512}, {"WGRAD_WG", 1024}, {"WGRAD_C1_TILES", 4},
    {"EIG_GRID", 32}, {"ROWS_BANDS", -1},
};

std::atomic<int> g_variant[V_COUNT];
std::once_flag g_variant_once;

void init_variants() {
  for (int i = 0; i < V_COUNT; ++i) {
    int v = kVariants[i].dflt;
    std::string env = std::string("SPECENH_") + kVariants[i].name;
    if (const char* s = std::getenv(env.c_str()); s && *s) v = std::atoi(s);
    g_variant[i].store(v, std::memory_order_relaxed);
  }
}

int variant_index(const char* name) {
  if (!name) return -1;
  if (std::strncmp(name, "SPECENH_", 8) == 0) name += 8;
  for (int i = 0; i < V_COUNT; ++i)
    if (std::strcmp(name, kVariants[i].name) == 0) return i;
  return -1;
}

constexpr int kMaxDevices = 64;
std::atomic<int> g_cus[kMaxDevices];

constexpr int kRing = 256;  // the calling thread's last kRing launches
thread_local const void* g_ring[kRing];
thread_local long long g_launches = 0;

}  // namespace

int variant(Variant v) {
  std::call_once(g_variant_once, init_variants);
  return g_variant[v].load(std::memory_order_relaxed);
}

int device_cus() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  int c = g_cus[dev].load(std::memory_order_relaxed);
  if (c > 0) return c;
  if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
    c = 256;
  g_cus[dev].store(c, std::memory_order_relaxed);  // same value from any racing thread
  return c;
}

void note_launch(const void* kernel) { g_ring[g_launches++ % kRing] = kernel; }

}  // namespace specenh

extern "C" {

int specenh_set_variant(const char* name, int value) {
  const int i = specenh::variant_index(name);
  if (i < 0) return specenh::set_error(SPECENH_EINVAL, std::string("unknown variant ") + (name ? name : "(null)"));
  std::call_once(specenh::g_variant_once, specenh::init_variants);
  specenh::g_variant[i].store(value, std::memory_order_relaxed);
  return SPECENH_OK;
}

int specenh_get_variant(const char* name, int* value) {
  const int i = specenh::variant_index(name);
  if (i < 0 || !value)
    return specenh::set_error(SPECENH_EINVAL, std::string("unknown variant ") + (name ? name : "(null)"));
  *value = specenh::variant((specenh::Variant)i);
  return SPECENH_OK;
}

long long specenh_launch_count(void) { return specenh::g_launches; }

const char* specenh_kernel_name_at(long long index) {
  using namespace specenh;
  if (index < 0 || index >= g_launches || index < g_launches - kRing) return "";
  const char* n = hipKernelNameRefByPtr(g_ring[index % kRing], nullptr);
  return n ? n : "";
}

int specenh_stream_wait(void* waiter, void* signaler, int device_scope) {
  using namespace specenh;
  constexpr int kEvents = 256;  // ring per device and fence kind: a reused event's earlier
                                 // waits were enqueued (and bound) long before
  static std::mutex mu;
  static hipEvent_t ring[kMaxDevices][2][kEvents] = {};
  static int next[kMaxDevices][2] = {};
  // The ring and the event belong to the signaler's device, not the thread's current one
  // (an engine on cuda:1 may run while the current device is 0).
  int dev = 0, cur = 0;
  if (hipStreamGetDevice((hipStream_t)signaler, &dev) != hipSuccess || dev < 0 ||
      dev >= kMaxDevices || hipGetDevice(&cur) != hipSuccess)
    return set_error(SPECENH_EHIP, "stream_wait: no device for the signaler stream");
  const int kind = device_scope ? 1 : 0;
  hipEvent_t ev;
  {
    std::lock_guard<std::mutex> lk(mu);
    hipEvent_t& e = ring[dev][kind][next[dev][kind]];
    next[dev][kind] = (next[dev][kind] + 1) % kEvents;
    if (!e) {
      const unsigned fl = hipEventDisableTiming | (device_scope ? hipEventDisableSystemFence : 0u);
      // events are created on the current device: switch to the signaler's for the creation
      const bool sw = cur != dev;
      if (sw && hipSetDevice(dev) != hipSuccess)
        return set_error(SPECENH_EHIP, "stream_wait: hipSetDevice");
      const hipError_t ce = hipEventCreateWithFlags(&e, fl);
      if (sw) (void)hipSetDevice(cur);
      if (ce != hipSuccess) {
        e = nullptr;
        return set_error(SPECENH_EHIP, "stream_wait: hipEventCreateWithFlags");
      }
    }
    ev = e;
  }
  if (hipEventRecord(ev, (hipStream_t)signaler) != hipSuccess ||
      hipStreamWaitEvent((hipStream_t)waiter, ev, 0) != hipSuccess)
    return set_error(SPECENH_EHIP, "stream_wait: record / wait");
  return SPECENH_OK;
}

const char* specenh_last_kernel_name(void) {
  return specenh_kernel_name_at(specenh::g_launches - 1);
}

}  // extern "C"

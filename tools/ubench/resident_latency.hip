// The floor of a resident real-time path: one wave of a kernel that stays on the GPU polls a
// mailbox in pinned host memory for a frame, and answers in mapped host words the host spins on -- against the
// launch-per-call floor (a kernel that only releases a word, flag_kernel: 6.3-6.6 us, profiles/r05_inline_frame.txt).
// Mailbox: N words of 8 bytes, (float sample, uint32 tag = request number); the host writes each word with one
// aligned 64-bit store and the wave reads each with one 64-bit system-scope load, so a word is old or new whole
// and the frame is complete when every tag is the request's (no ordering between words is assumed).
//   A  the wave reads the whole mailbox every poll;
//   B  it polls the first word only, then reads the whole mailbox (one more PCIe round trip);
//   P  as A with two polls in flight; W as P, the answer written through without the system-scope release;
//   Q  as A with four polls in flight;
//   L  a one-wave kernel launch per call that reads the same mailbox and answers the same way (the product's
//      protocol today, minus its extraction).
// The answer: the frame's sum (lane partial sums, DPP-free shuffles) in one host word, then the request number.
// Every wave exits: on the host's stop word, or 2 s after its last request.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ubench/resident_latency tools/ubench/resident_latency.hip
// usage: resident_latency [N] [calls]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint64_t sys_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the frame's words, lane l holding words l, l + 64, ... (W per lane, every load issued before any is
// used); true when every tag is `seq`
template <int W>
__device__ __forceinline__ bool read_frame(const uint64_t* mail, uint32_t seq, float& sum) {
  uint64_t w[W];
#pragma unroll
  for (int k = 0; k < W; ++k) w[k] = sys_load(mail + threadIdx.x + 64 * k);
  uint32_t bad = 0;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    bad |= (uint32_t)(w[k] >> 32) ^ seq;
    s += __uint_as_float((uint32_t)w[k]);
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  sum = s;
  return __all(bad == 0);
}

__device__ __forceinline__ void answer(uint32_t* out, float sum, uint32_t seq) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(out + 1, __float_as_uint(sum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int W, bool HEAD_FIRST>
__global__ void server(const uint64_t* mail, uint32_t* out, const uint32_t* stop, uint32_t* polls) {
  uint32_t seq = 1, npoll = 0;
  unsigned long long last = wall_clock64();
  const unsigned long long limit = 200000000ull;  // 2 s of the 100 MHz clock
  for (;;) {
    float sum = 0.0f;
    bool ok;
    if (HEAD_FIRST) {
      ok = (uint32_t)(sys_load(mail) >> 32) == seq;
      if (ok) ok = read_frame<W>(mail, seq, sum);  // (a partly written frame: polled again)
    } else {
      ok = read_frame<W>(mail, seq, sum);
    }
    ++npoll;
    if (ok) {
      answer(out, sum, seq);
      ++seq;
      last = wall_clock64();
      continue;
    }
    if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
    if (wall_clock64() - last > limit) break;
  }
  if (threadIdx.x == 0) polls[0] = npoll;
}

// P: D polls in flight -- the next ones are issued before the oldest is checked (vector loads return in
// issue order), so a posted frame is seen one round trip after it lands instead of up to two
template <int W>
__device__ __forceinline__ void issue(uint64_t (&w)[W], const uint64_t* mail) {
#pragma unroll
  for (int k = 0; k < W; ++k) w[k] = sys_load(mail + threadIdx.x + 64 * k);
}
template <int W>
__device__ __forceinline__ bool check(const uint64_t (&w)[W], uint32_t seq, float& sum) {
  uint32_t bad = 0;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < W; ++k) {
    bad |= (uint32_t)(w[k] >> 32) ^ seq;
    s += __uint_as_float((uint32_t)w[k]);
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  sum = s;
  return __all(bad == 0);
}
// the answer without the system-scope release (no L2 write-back): both words written through (system-scope
// relaxed stores), the second after the first's acknowledgement (s_waitcnt vmcnt(0))
__device__ __forceinline__ void answer_wt(uint32_t* out, float sum, uint32_t seq) {
  if (threadIdx.x == 0) {
    __hip_atomic_store(out + 1, __float_as_uint(sum), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_s_waitcnt(0);
    __hip_atomic_store(out, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int W, bool WT = false>
__global__ void server_pipe(const uint64_t* mail, uint32_t* out, const uint32_t* stop, uint32_t* polls) {
  uint32_t seq = 1, npoll = 0;
  unsigned long long last = wall_clock64();
  const unsigned long long limit = 200000000ull;
  uint64_t a[W], b[W];
  issue<W>(a, mail);
  for (;;) {
    float sum;
    issue<W>(b, mail);
    if (check<W>(a, seq, sum)) {
      if (WT) answer_wt(out, sum, seq);
      else answer(out, sum, seq);
      ++seq;
      last = wall_clock64();
    }
    issue<W>(a, mail);
    if (check<W>(b, seq, sum)) {
      if (WT) answer_wt(out, sum, seq);
      else answer(out, sum, seq);
      ++seq;
      last = wall_clock64();
    }
    npoll += 2;
    if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
    if (wall_clock64() - last > limit) break;
  }
  if (threadIdx.x == 0) polls[0] = npoll;
}

// Q: four reads in flight (a round trip's worth of reads issued at a quarter of it apart)
template <int W>
__global__ void server_pipe4(const uint64_t* mail, uint32_t* out, const uint32_t* stop, uint32_t* polls) {
  uint32_t seq = 1;
  unsigned long long last = wall_clock64();
  const unsigned long long limit = 200000000ull;
  uint64_t a[W], b[W], c[W], d[W];
  issue<W>(a, mail);
  issue<W>(b, mail);
  issue<W>(c, mail);
  for (;;) {
    float sum;
    issue<W>(d, mail);
    if (check<W>(a, seq, sum)) { answer(out, sum, seq); ++seq; last = wall_clock64(); }
    issue<W>(a, mail);
    if (check<W>(b, seq, sum)) { answer(out, sum, seq); ++seq; last = wall_clock64(); }
    issue<W>(b, mail);
    if (check<W>(c, seq, sum)) { answer(out, sum, seq); ++seq; last = wall_clock64(); }
    issue<W>(c, mail);
    if (check<W>(d, seq, sum)) { answer(out, sum, seq); ++seq; last = wall_clock64(); }
    if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) break;
    if (wall_clock64() - last > limit) break;
  }
  if (threadIdx.x == 0) polls[0] = seq;
}

template <int W>
__global__ void one_shot(const uint64_t* mail, uint32_t* out, uint32_t seq) {
  float sum = 0.0f;
  for (int k = 0; k < 1000000 && !read_frame<W>(mail, seq, sum); ++k) {
  }
  answer(out, sum, seq);
}

static double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static void post(volatile uint64_t* mail, int n, uint32_t seq) {
  for (int i = 0; i < n; ++i) {
    const float x = (float)((i * 7919 + seq) % 2001 - 1000) / 1000.0f;
    uint32_t b;
    memcpy(&b, &x, 4);
    mail[i] = ((uint64_t)seq << 32) | b;
  }
}

static void report(const char* name, std::vector<double> v) {
  std::sort(v.begin(), v.end());
  printf("\"%s_us\": %.2f, \"%s_p90_us\": %.2f, ", name, v[v.size() / 2], name, v[(size_t)(0.9 * (v.size() - 1))]);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 512;
  if (n != 512 && n != 1024) return 2;
  const int calls = argc > 2 ? atoi(argv[2]) : 3000;
  uint64_t *hmail, *dmail;
  uint32_t *hout, *dout, *hstop, *dstop, *dpolls;
  CK(hipHostMalloc((void**)&hmail, n * 8, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&hout, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&hstop, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&dmail, hmail, 0));
  CK(hipHostGetDevicePointer((void**)&dout, hout, 0));
  CK(hipHostGetDevicePointer((void**)&dstop, hstop, 0));
  CK(hipMalloc((void**)&dpolls, 64));
  volatile uint64_t* vmail = hmail;
  volatile uint32_t* vout = hout;
  volatile uint32_t* vstop = hstop;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  printf("{\"n\": %d, \"calls\": %d, ", n, calls);
  for (int mode = 0; mode < 6; ++mode) {
    memset(hmail, 0, n * 8);
    *vout = 0;
    *vstop = 0;
    std::vector<double> t;
    if (mode == 3) {
      if (n == 512) server_pipe<8><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
      else server_pipe<16><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
    } else if (mode == 5) {
      if (n == 512) server_pipe4<8><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
      else server_pipe4<16><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
    } else if (mode == 4) {
      if (n == 512) server_pipe<8, true><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
      else server_pipe<16, true><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
    } else if (mode < 2) {
      if (n == 512) {
        if (mode == 0) server<8, false><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
        else server<8, true><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
      } else {
        if (mode == 0) server<16, false><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
        else server<16, true><<<1, 64, 0, s>>>(dmail, dout, dstop, dpolls);
      }
      CK(hipGetLastError());
    }
    for (uint32_t seq = 1; seq <= (uint32_t)calls + 50; ++seq) {
      const double t0 = now_us();
      post(vmail, n, seq);
      if (mode == 2 && n == 512) one_shot<8><<<1, 64, 0, s>>>(dmail, dout, seq);
      if (mode == 2 && n == 1024) one_shot<16><<<1, 64, 0, s>>>(dmail, dout, seq);
      const double tw = now_us();
      while (*vout != seq) {
        if (now_us() - tw > 1e6) {
          fprintf(stderr, "no answer to request %u (mode %d)\n", seq, mode);
          *vstop = 1;
          CK(hipStreamSynchronize(s));
          return 1;
        }
      }
      const double t1 = now_us();
      if (seq > 50) t.push_back(t1 - t0);
    }
    *vstop = 1;
    CK(hipStreamSynchronize(s));
    report(mode == 0 ? "resident_full_poll" : mode == 1 ? "resident_head_poll" : mode == 2 ? "launch_per_call"
           : mode == 3 ? "resident_pipelined_poll" : mode == 4 ? "resident_pipelined_poll_write_through"
           : "resident_four_reads_in_flight", t);
  }
  printf("\"post_only_us\": ");
  {
    const double t0 = now_us();
    for (int k = 0; k < 1000; ++k) post(vmail, n, 7);
    printf("%.3f}\n", (now_us() - t0) / 1000);
  }
  return 0;
}

// Where a one-frame host call's time goes (the real-time path, plan.cpp extract_host_small):
// the extraction launched on device-mapped pinned host buffers, then
//   A  hipStreamSynchronize (what extract_host_small does),
//   B  a host spin on the mapped output words (sentinel bits -> value), then the stream sync,
//   C  an empty kernel + hipStreamSynchronize (the launch and wake-up floor),
//   E  a busy loop on hipStreamQuery, F  an event and a busy loop on hipEventQuery,
//   D  the kernel's own duration between two events, G  the same on device-resident frames and outputs,
//   K  mgx_extract_host on a MGX_FLAG_RESIDENT plan (the frame to a resident workgroup through a mailbox);
//   H  a kernel that only releases a sequence number to a mapped host word, the host spinning on it (the
//      protocol's floor), H2 the same with 2,480 bytes of kernel arguments, H3 the same through
//      hipModuleLaunchKernel with pre-packed arguments, I  mgx_extract_host itself, J  one hipSetDevice call
//      (0.07 us: the small path's two per call cost nothing measurable).
// Build: hipcc --offload-arch=gfx950 -O2 -I include -o tools/ubench/small_latency tools/ubench/small_latency.hip \
//          -L meyda_amd -lmeyda_gpu -Wl,-rpath,$PWD/meyda_amd
// usage: small_latency [N] [calls]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#include "meyda_gpu.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void empty_kernel() {}
// H: the floor of the small host path's protocol -- a kernel that only releases a sequence number to a
// mapped host word (as done_signal), the host spinning on it; H2 the same with 2,480 bytes of kernel
// arguments (KernelArgsInline's size: what a one-frame launch at N = 512 passes)
__global__ void flag_kernel(uint32_t* flag, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
struct BigArgs {
  uint32_t* flag;
  uint32_t seq;
  float pad[616];
};
__global__ void flag_kernel_big(BigArgs a) {
  if (threadIdx.x == 0) __hip_atomic_store(a.flag, a.seq + (uint32_t)a.pad[threadIdx.x], __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 512;
  const int calls = argc > 2 ? atoi(argv[2]) : 2000;
  mgx_plan_desc d;
  mgx_plan_desc_init(&d);
  d.buffer_size = (uint32_t)n;
  mgx_plan* p = nullptr;
  if (mgx_plan_create(&d, &p) != MGX_OK) {
    fprintf(stderr, "plan: %s\n", mgx_last_error());
    return 1;
  }
  float *hin, *hout, *din, *dout;
  CK(hipHostMalloc((void**)&hin, n * sizeof(float), hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&hout, 256, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&din, hin, 0));
  CK(hipHostGetDevicePointer((void**)&dout, hout, 0));
  for (int i = 0; i < n; ++i) hin[i] = (float)((i * 7919) % 2001 - 1000) / 1000.0f;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  mgx_outputs o;
  memset(&o, 0, sizeof(o));
  o.scalars[MGX_RMS] = dout;
  o.scalars[MGX_SPECTRAL_CENTROID] = dout + 16;
  volatile uint32_t* w0 = reinterpret_cast<volatile uint32_t*>(hout);
  volatile uint32_t* w1 = reinterpret_cast<volatile uint32_t*>(hout + 16);
  const uint32_t kSentinel = 0xFFBADBADu;  // a NaN payload the kernel never writes for finite input
  // G: the same kernel on device-resident frames and outputs (no PCIe in the kernel's chain)
  float *gin, *gout;
  CK(hipMalloc((void**)&gin, n * sizeof(float)));
  CK(hipMalloc((void**)&gout, 256));
  CK(hipMemcpy(gin, hin, n * sizeof(float), hipMemcpyHostToDevice));
  mgx_outputs og;
  memset(&og, 0, sizeof(og));
  og.scalars[MGX_RMS] = gout;
  og.scalars[MGX_SPECTRAL_CENTROID] = gout + 16;
  std::vector<double> tg;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> ta, tb, tc, td, tl, te, tf, th, th2, th3, ti;
  uint32_t* hflag = nullptr;
  uint32_t* dflag = nullptr;
  CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
  volatile uint32_t* vflag = hflag;
  hipFunction_t fk;
  CK(hipGetFuncBySymbol(&fk, reinterpret_cast<const void*>(flag_kernel)));
  *vflag = 0;
  uint32_t seq = 0;
  BigArgs big;
  memset(&big, 0, sizeof(big));
  big.flag = dflag;
  // I: the product's one-frame host call (mgx_extract_host: pinned buffers, the frame in the kernel arguments
  // at N <= 512, the completion word) for the same two features
  double hrms[1], hcen[1];
  mgx_plan_desc dh;
  mgx_plan_desc_init(&dh);
  dh.buffer_size = (uint32_t)n;
  dh.scalar_f64 = 1;
  mgx_plan* ph = nullptr;
  if (mgx_plan_create(&dh, &ph) != MGX_OK) return 1;
  mgx_outputs oh;
  memset(&oh, 0, sizeof(oh));
  oh.scalars[MGX_RMS] = hrms;
  oh.scalars[MGX_SPECTRAL_CENTROID] = hcen;
  for (int it = 0; it < calls + 50; ++it) {
    // A: launch + stream synchronise
    double t0 = now_us();
    if (mgx_extract_device(p, din, 1, &o, s) != MGX_OK) return 1;
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    double t2 = now_us();
    // B: launch + spin on the mapped outputs, then the stream sync (outside the time)
    *w0 = kSentinel;
    *w1 = kSentinel;
    double t3 = now_us();
    if (mgx_extract_device(p, din, 1, &o, s) != MGX_OK) return 1;
    while (*w0 == kSentinel || *w1 == kSentinel) {
    }
    double t4 = now_us();
    CK(hipStreamSynchronize(s));
    // E: launch + a busy loop on hipStreamQuery
    double t7 = now_us();
    if (mgx_extract_device(p, din, 1, &o, s) != MGX_OK) return 1;
    while (hipStreamQuery(s) == hipErrorNotReady) {
    }
    double t8 = now_us();
    // F: launch + event record + a busy loop on hipEventQuery
    double t9 = now_us();
    if (mgx_extract_device(p, din, 1, &o, s) != MGX_OK) return 1;
    CK(hipEventRecord(e1, s));
    while (hipEventQuery(e1) == hipErrorNotReady) {
    }
    double t10 = now_us();
    // C: empty kernel
    double t5 = now_us();
    empty_kernel<<<1, 64, 0, s>>>();
    CK(hipStreamSynchronize(s));
    double t6 = now_us();
    // H / H2: the flag kernel's round trip
    double t11 = now_us();
    flag_kernel<<<1, 64, 0, s>>>(dflag, ++seq);
    while (*vflag != seq) {
    }
    double t12 = now_us();
    big.seq = ++seq;
    double t13 = now_us();
    flag_kernel_big<<<1, 64, 0, s>>>(big);
    while (*vflag != seq) {
    }
    double t14 = now_us();
    CK(hipStreamSynchronize(s));
    // H3: the flag kernel through hipModuleLaunchKernel with the arguments pre-packed (HIP_LAUNCH_PARAM_BUFFER_*)
    struct {
      uint32_t* flag;
      uint32_t seq;
      uint32_t pad;
    } packed = {dflag, ++seq, 0};
    size_t psize = sizeof(packed);
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &packed, HIP_LAUNCH_PARAM_BUFFER_SIZE, &psize, HIP_LAUNCH_PARAM_END};
    double t17 = now_us();
    CK(hipModuleLaunchKernel(fk, 1, 1, 1, 64, 1, 1, 0, s, nullptr, extra));
    while (*vflag != seq) {
    }
    double t18 = now_us();
    CK(hipStreamSynchronize(s));
    // I: the product's host call
    double t15 = now_us();
    if (mgx_extract_host(ph, hin, 1, &oh) != MGX_OK) return 1;
    double t16 = now_us();
    // D: kernel duration
    CK(hipEventRecord(e0, s));
    if (mgx_extract_device(p, din, 1, &o, s) != MGX_OK) return 1;
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventRecord(e0, s));
    if (mgx_extract_device(p, gin, 1, &og, s) != MGX_OK) return 1;
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float msg = 0;
    CK(hipEventElapsedTime(&msg, e0, e1));
    if (it >= 50) {
      tg.push_back(msg * 1e3);
      ta.push_back(t2 - t0);
      tl.push_back(t1 - t0);
      tb.push_back(t4 - t3);
      tc.push_back(t6 - t5);
      td.push_back(ms * 1e3);
      te.push_back(t8 - t7);
      tf.push_back(t10 - t9);
      th.push_back(t12 - t11);
      th2.push_back(t14 - t13);
      ti.push_back(t16 - t15);
      th3.push_back(t18 - t17);
    }
  }
  // K: mgx_extract_host on a plan with MGX_FLAG_RESIDENT (one workgroup stays on the device, polling a mailbox
  // in pinned host memory): the same frame and features, after the loop above (the launch-per-call plans idle)
  std::vector<double> tk;
  double krms[1], kcen[1];
  {
    mgx_plan_desc dr = dh;
    dr.flags |= MGX_FLAG_RESIDENT;
    mgx_plan* pr = nullptr;
    if (mgx_plan_create(&dr, &pr) != MGX_OK) {
      fprintf(stderr, "resident plan: %s\n", mgx_last_error());
      return 1;
    }
    mgx_outputs orr;
    memset(&orr, 0, sizeof(orr));
    orr.scalars[MGX_RMS] = krms;
    orr.scalars[MGX_SPECTRAL_CENTROID] = kcen;
    for (int it = 0; it < calls + 50; ++it) {
      const double t0 = now_us();
      if (mgx_extract_host(pr, hin, 1, &orr) != MGX_OK) {
        fprintf(stderr, "resident call: %s\n", mgx_last_error());
        return 1;
      }
      const double t1 = now_us();
      if (it >= 50) tk.push_back(t1 - t0);
    }
    if (krms[0] != hrms[0] || kcen[0] != hcen[0]) {
      fprintf(stderr, "resident outputs differ: %.17g %.17g vs %.17g %.17g\n", krms[0], kcen[0], hrms[0], hcen[0]);
      return 1;
    }
    mgx_plan_destroy(pr);
  }
  std::sort(tk.begin(), tk.end());
  printf("{\"extract_host_resident_us\": %.2f, \"extract_host_resident_p90_us\": %.2f, \"extract_host_resident_min_us\": %.2f}\n",
         tk[tk.size() / 2], tk[(size_t)(0.9 * (tk.size() - 1))], tk[0]);
  // J: the cost of one hipSetDevice call (the small host path makes two per call)
  double tj0 = now_us();
  for (int i = 0; i < 20000; ++i) CK(hipSetDevice(0));
  const double set_device_us = (now_us() - tj0) / 20000;
  printf("{\"set_device_us\": %.3f}\n", set_device_us);
  printf("{\"n\": %d, \"calls\": %d, \"launch_sync_us\": %.2f, \"launch_call_us\": %.2f, \"launch_spin_us\": %.2f, "
         "\"launch_stream_query_us\": %.2f, \"launch_event_query_us\": %.2f, "
         "\"empty_kernel_sync_us\": %.2f, \"kernel_event_us\": %.2f, \"kernel_event_device_io_us\": %.2f, "
         "\"flag_kernel_spin_us\": %.2f, \"flag_kernel_2480B_args_spin_us\": %.2f, \"flag_kernel_module_launch_spin_us\": %.2f, "
         "\"extract_host_us\": %.2f, "
         "\"rms\": %.9g, \"centroid\": %.9g}\n",
         n, calls, median(ta), median(tl), median(tb), median(te), median(tf), median(tc), median(td), median(tg), median(th),
         median(th2), median(th3), median(ti), hout[0], hout[16]);
  mgx_plan_destroy(p);
  return 0;
}

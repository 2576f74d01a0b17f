// tools/hop_latency.hip -- latency of one progress-word hand-off between two
// workgroups, as the frame-interleaved group and a row shard would
// pay it, measured on one MI355X ("Hop latency").
//
// One hop = the producer's payload stores (the deblock chunk's words, or none),
// every storing wave's s_waitcnt vmcnt(0), the workgroup barrier, thread 0's
// release fence and the progress word's store; then the consumer's poll sees
// the word, its acquire fence, and its loads of the payload.  Two workgroups
// ping-pong N times (ping: store word i, poll pong == i; pong: poll word i,
// store pong = i); one hop = the round trip / 2, timed by s_memrealtime
// (100 MHz) on the ping side.
//
// Modes:
//   local <scope> <xcd> <payload_bytes> <iters>   one process, one kernel of
//       two workgroups; scope "agent" (coarse-grained memory, agent-scope
//       fences and sc1 accesses: one context's hand-offs) or "system"
//       (fine-grained memory, system scope: a group member's); xcd "same"
//       (blocks 0 and 8: one XCD under round-robin dispatch) or "cross"
//       (blocks 0 and 1).
//   ping <file> <payload_bytes> <iters>   two processes on one device: the
//   pong <file> <payload_bytes> <iters>   buffers are fine-grained, exported by
//       ping through an IPC handle written to <file> (pong imports it and
//       creates <file>.ready), system scope throughout -- the cross-process
//       path of a group member, minus the xGMI link.
// Every poll is bounded (2 s), so a lost partner ends the run with an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                             \
    }                                                                                      \
  } while (0)

// Buffer layout (uint32 words): [0] ping word, [64] pong word, [128..) the ping
// side's payload, then the pong side's payload; timing results after both.
constexpr int kPing = 0, kPong = 64, kPay = 128;
constexpr uint64_t kLimit = 200000000ull;  // 2 s of s_memrealtime

struct Args {
  uint32_t* buf;
  uint32_t* times;  // ping side: round trips in 10 ns ticks
  int iters, pay_words, sys, role_of_block0;  // role: 0 ping, 1 pong
  int blocks_apart;
};

__device__ __forceinline__ uint32_t poll_load(const uint32_t* p, int sys) {
  return sys ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
             : __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One side's hand-off: payload stores, drain, barrier, release, word.
__device__ __forceinline__ void publish(uint32_t* word, uint32_t* pay, int pay_words, uint32_t v, int sys) {
  for (int k = threadIdx.x; k < pay_words; k += blockDim.x) {
    if (sys)
      __hip_atomic_store(pay + k, v + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      __hip_atomic_store(pay + k, v + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (sys) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_store(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The other side: poll the word (thread 0), acquire, barrier, payload loads.
// Returns false on a timeout.
__device__ __forceinline__ bool consume(const uint32_t* word, const uint32_t* pay, int pay_words, uint32_t v,
                                        int sys, int* lds_ok, uint32_t* sink) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while (poll_load(word, sys) != v) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > kLimit) {
        ok = 0;
        break;
      }
    }
    if (sys)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    else
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *lds_ok = ok;
  }
  __syncthreads();
  uint32_t acc = 0;
  for (int k = threadIdx.x; k < pay_words; k += blockDim.x) acc += pay[k] - (v + k);
  if (acc) atomicAdd(sink, 1u);  // a payload word older than the word: counted, never expected
  const bool ok = *lds_ok != 0;
  __syncthreads();
  return ok;
}

__global__ void __launch_bounds__(256) k_hop(Args a) {
  __shared__ int ok_word;
  int role;
  if (a.role_of_block0 < 0) {  // local mode: block 0 pings, block blocks_apart pongs
    if (blockIdx.x == 0) role = 0;
    else if ((int)blockIdx.x == a.blocks_apart) role = 1;
    else return;
  } else {
    role = a.role_of_block0;
  }
  uint32_t* ping = a.buf + kPing;
  uint32_t* pong = a.buf + kPong;
  uint32_t* pay_ping = a.buf + kPay;
  uint32_t* pay_pong = a.buf + kPay + a.pay_words;
  uint32_t* sink = a.buf + kPay + 2 * a.pay_words;
  for (int i = 1; i <= a.iters; i++) {
    if (role == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      publish(ping, pay_ping, a.pay_words, (uint32_t)i, a.sys);
      if (!consume(pong, pay_pong, a.pay_words, (uint32_t)i, a.sys, &ok_word, sink)) {
        if (threadIdx.x == 0) a.times[0] = 0xFFFFFFFFu;
        return;
      }
      if (threadIdx.x == 0) a.times[i] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
    } else {
      if (!consume(ping, pay_ping, a.pay_words, (uint32_t)i, a.sys, &ok_word, sink)) return;
      publish(pong, pay_pong, a.pay_words, (uint32_t)i, a.sys);
    }
  }
}

// Stale-line probe (mode "stale"): can a workgroup on one XCD, after an
// agent-scope acquire that observed a producer's flag, still read a line its
// XCD's L2 cached before the producer (on another XCD) wrote it?  Per trial k
// on its own 128-byte line: the consumer loads the line (plain) and raises
// `loaded`; the producer, seeing it, stores the line's word -- sc1 (write-
// through, as the engine's coefficient stores) or plain followed by a release
// fence -- drains and raises `written` (release); the consumer acquires and
// reloads the word plainly and with an sc1 load.  Counts of stale values.
__global__ void __launch_bounds__(64) k_stale(uint32_t* data, uint32_t* flags, uint32_t* out, int trials,
                                              int plain_store) {
  const bool producer = blockIdx.x == 0, consumer = blockIdx.x == 1;
  if (!(producer || consumer) || threadIdx.x != 0) return;
  uint32_t stale_plain = 0, stale_sc1 = 0, timeouts = 0, sink = 0;
  for (int k = 0; k < trials; k++) {
    uint32_t* word = data + (size_t)k * 32;  // one line per trial
    const uint32_t v = 0x5A000000u | (uint32_t)k;
    if (consumer) {
      sink += *(volatile uint32_t*)word;  // the line into this XCD's L1/L2 (value 0)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(flags + 0, (uint32_t)(k + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(flags + 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (uint32_t)(k + 1))
        if (__builtin_amdgcn_s_memrealtime() - t0 > kLimit) { timeouts++; k = trials; break; }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const uint32_t a = *(volatile uint32_t*)word;
      const uint32_t b = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      stale_plain += a != v;
      stale_sc1 += b != v;
    } else {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(flags + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != (uint32_t)(k + 1))
        if (__builtin_amdgcn_s_memrealtime() - t0 > kLimit) { timeouts++; k = trials; break; }
      if (plain_store) {
        *(volatile uint32_t*)word = v;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      } else {
        __hip_atomic_store(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(flags + 32, (uint32_t)(k + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (consumer) out[0] = stale_plain, out[1] = stale_sc1, out[2] = sink, out[4] = timeouts;
  else out[3] = timeouts;
}

static size_t buf_bytes(int pay_words) { return (size_t)(kPay + 2 * pay_words + 64) * 4; }

static void report(const char* what, const uint32_t* t, int iters, int pay_bytes) {
  if (t[0] == 0xFFFFFFFFu) {
    printf("{\"mode\": \"%s\", \"error\": \"a poll timed out\"}\n", what);
    exit(3);
  }
  std::vector<double> us;
  for (int i = 1 + iters / 10; i <= iters; i++) us.push_back(t[i] * 0.01 / 2.0);  // one hop, warm-up dropped
  std::sort(us.begin(), us.end());
  double sum = 0;
  for (double x : us) sum += x;
  printf("{\"mode\": \"%s\", \"payload_bytes\": %d, \"hops\": %zu, \"hop_us_median\": %.3f, \"hop_us_mean\": %.3f, "
         "\"hop_us_p10\": %.3f, \"hop_us_p90\": %.3f}\n",
         what, pay_bytes, us.size(), us[us.size() / 2], sum / us.size(), us[us.size() / 10],
         us[us.size() * 9 / 10]);
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: hop_latency local agent|system same|cross <payload_bytes> <iters>\n"
                    "       hop_latency ping|pong <file> <payload_bytes> <iters>\n");
    return 1;
  }
  const std::string mode = argv[1];
  if (mode == "local" && argc == 6) {
    const bool sys = std::string(argv[2]) == "system";
    const bool same = std::string(argv[3]) == "same";
    const int pay = atoi(argv[4]) / 4, iters = atoi(argv[5]);
    Args a{};
    const size_t bytes = buf_bytes(pay);
    if (sys)
      CK(hipExtMallocWithFlags((void**)&a.buf, bytes, hipDeviceMallocFinegrained));
    else
      CK(hipMalloc(&a.buf, bytes));
    CK(hipMemset(a.buf, 0, bytes));
    CK(hipMalloc(&a.times, (iters + 1) * 4));
    CK(hipMemset(a.times, 0, (iters + 1) * 4));
    a.iters = iters, a.pay_words = pay, a.sys = sys, a.role_of_block0 = -1, a.blocks_apart = same ? 8 : 1;
    hipLaunchKernelGGL(k_hop, dim3(a.blocks_apart + 1), dim3(256), 0, 0, a);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> t(iters + 1);
    CK(hipMemcpy(t.data(), a.times, (iters + 1) * 4, hipMemcpyDeviceToHost));
    const std::string what = std::string("local-") + argv[2] + "-" + argv[3] + "-xcd";
    report(what.c_str(), t.data(), iters, pay * 4);
    return 0;
  }
  if (mode == "stale" && argc == 4) {  // stale <sc1|plain> <trials>
    const int plain = std::string(argv[2]) == "plain", trials = atoi(argv[3]);
    uint32_t *data, *flags, *out;
    CK(hipMalloc(&data, (size_t)trials * 128));
    CK(hipMemset(data, 0, (size_t)trials * 128));
    CK(hipMalloc(&flags, 256));
    CK(hipMemset(flags, 0, 256));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(out, 0, 64));
    hipLaunchKernelGGL(k_stale, dim3(2), dim3(64), 0, 0, data, flags, out, trials, plain);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    uint32_t o[5];
    CK(hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost));
    printf("{\"mode\": \"stale-%s-store\", \"trials\": %d, \"stale_plain_loads\": %u, \"stale_sc1_loads\": %u, "
           "\"timeouts\": %u}\n",
           plain ? "plain+release" : "sc1", trials, o[0], o[1], o[3] + o[4]);
    return 0;
  }
  if ((mode == "ping" || mode == "pong") && argc == 5) {
    const std::string file = argv[2];
    const int pay = atoi(argv[3]) / 4, iters = atoi(argv[4]);
    const size_t bytes = buf_bytes(pay);
    Args a{};
    a.iters = iters, a.pay_words = pay, a.sys = 1, a.role_of_block0 = mode == "ping" ? 0 : 1;
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(60);
    if (mode == "ping") {
      CK(hipExtMallocWithFlags((void**)&a.buf, bytes, hipDeviceMallocFinegrained));
      CK(hipMemset(a.buf, 0, bytes));
      hipIpcMemHandle_t h;
      CK(hipIpcGetMemHandle(&h, a.buf));
      FILE* f = fopen((file + ".tmp").c_str(), "wb");
      fwrite(&h, sizeof(h), 1, f);
      fclose(f);
      rename((file + ".tmp").c_str(), file.c_str());
      for (;;) {  // the partner has imported the buffer
        if (FILE* r = fopen((file + ".ready").c_str(), "rb")) {
          fclose(r);
          break;
        }
        if (std::chrono::steady_clock::now() > deadline) {
          fprintf(stderr, "ping: no partner\n");
          return 3;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
      CK(hipMalloc(&a.times, (iters + 1) * 4));
      CK(hipMemset(a.times, 0, (iters + 1) * 4));
    } else {
      hipIpcMemHandle_t h;
      for (;;) {
        if (FILE* f = fopen(file.c_str(), "rb")) {
          const size_t n = fread(&h, sizeof(h), 1, f);
          fclose(f);
          if (n == 1) break;
        }
        if (std::chrono::steady_clock::now() > deadline) {
          fprintf(stderr, "pong: no handle\n");
          return 3;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
      CK(hipIpcOpenMemHandle((void**)&a.buf, h, hipIpcMemLazyEnablePeerAccess));
      CK(hipMalloc(&a.times, 4));
      FILE* r = fopen((file + ".ready").c_str(), "wb");
      fclose(r);
    }
    hipLaunchKernelGGL(k_hop, dim3(1), dim3(256), 0, 0, a);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    if (mode == "ping") {
      std::vector<uint32_t> t(iters + 1);
      CK(hipMemcpy(t.data(), a.times, (iters + 1) * 4, hipMemcpyDeviceToHost));
      report("cross-process-system", t.data(), iters, pay * 4);
    } else {
      CK(hipIpcCloseMemHandle(a.buf));
    }
    return 0;
  }
  fprintf(stderr, "bad arguments\n");
  return 1;
}

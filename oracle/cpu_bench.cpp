// cpu_bench.cpp -- the CPU baseline of bench.py: the
// REFERENCE's own code timed on this host's cores.  TEST/MEASUREMENT
// INFRASTRUCTURE ONLY -- never part of the product path.
//
// Built by oracle/Makefile into _ref/cpu_bench (linked against
// _ref/libref_filter.so, the reference's src/filter.cpp compiled where it
// lies) or into cpu_bench_port (linked against liboracle.so, the C
// restatement) when the reference is not present.
//
//   cpu_bench <kernel> <block> <seconds> <threads>
//       one config's kernel on independent synthetic streams, one stream per
//       std::thread, one per core of the CPU share (<threads> = 0), pinned one
//       per core when the whole affinity set is the share; block after block
//       with the state carried, until <seconds> have passed (at least one
//       block).  <kernel>:
//         frontend  the mode-0 front end (src/project.cpp:86-90: FIR+dec10 on
//                   I and Q, then fmDemodArctan); unit = IQ pairs (cfg2, cfg4)
//         resample  resampleBlockConvolveFIR 147/800 with 151 taps per phase
//                   (src/filter.cpp:142-173, impulseResponseLPF(240e3*147,
//                   16e3, 22197, 147), state 150); unit = input samples (cfg3)
//         fir1024   blockConvolveFIR with the 1024-tap LPF on I and Q
//                   (src/filter.cpp:66-83, state 1023); unit = IQ pairs (cfg5)
//       Prints {"pairs":..., "seconds":..., "threads":...} (pairs = units).
//   cpu_bench program <project_binary> <blocks> <procs> [mono|stereo]
//       BASELINE config 1: `<project_binary> 0 mono` (the reference program,
//       src/project.cpp; `stereo` for its stereo path) run as <procs>
//       concurrent child processes, each fed <blocks> 102,400-byte u8 IQ
//       blocks on stdin (51,200 pairs, src/project.cpp:188) while its PCM is
//       drained from stdout.  Wall clock from spawn to the last exit.  Prints
//       {"pairs":..., "seconds":..., "procs":..., "pcm_bytes":...}.
//   cpu_bench cores
//       Prints the CPU share: the affinity set (sched_getaffinity) capped by
//       the cgroup CPU quota and OMP_NUM_THREADS (cpu_share below).
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <signal.h>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef CPU_BENCH_PORT
extern "C" {
// oracle/_ref/libref_filter.so (ref_shim.cpp): the reference's own
// src/filter.cpp behind a block-after-block front-end runner
void* ref_front_new(const float* h, int nh, int ns);
void ref_front_free(void* p);
long ref_front_run(void* p, int D, const float* I, const float* Q, long n, float* demod);
long ref_taps_lpf(float Fs, float Fc, unsigned short T, int up, float* h);
void* ref_resample_new(int up, int down, const float* h, int nh, int ns);
void ref_resample_free(void* p);
long ref_resample_run(void* p, const float* x, long n, float* y);
void* ref_block_new(const float* h, int nh, int ns);
void ref_block_free(void* p);
long ref_block_run(void* p, const float* I, const float* Q, long n, float* yi, float* yq);
}
#else
// the C restatement (liboracle.so) when the reference was not built
#include "sdr_oracle.h"
namespace {
struct PortFront {
  std::vector<float> h, si, sq, yi, yq;
  float pi = 0, pq = 0;
};
}  // namespace
static void* ref_front_new(const float* h, int nh, int ns) {
  auto* f = new PortFront;
  f->h.assign(h, h + nh);
  f->si.assign(ns, 0.0f);
  f->sq.assign(ns, 0.0f);
  return f;
}
static void ref_front_free(void* p) { delete static_cast<PortFront*>(p); }
static long ref_front_run(void* p, int D, const float* I, const float* Q, long n, float* demod) {
  auto* f = static_cast<PortFront*>(p);
  f->yi.resize(n / D);
  f->yq.resize(n / D);
  return or_frontend(D, I, Q, n, f->h.data(), (int)f->h.size(), f->si.data(), f->sq.data(), (int)f->si.size(),
                     &f->pi, &f->pq, f->yi.data(), f->yq.data(), demod);
}
static long ref_taps_lpf(float Fs, float Fc, unsigned short T, int up, float* h) { return or_taps_lpf(Fs, Fc, T, up, h); }
namespace {
struct PortResample {
  int up, down;
  std::vector<float> h, st, y;
};
struct PortBlock {
  std::vector<float> h, si, sq, yi, yq;
};
}  // namespace
static void* ref_resample_new(int up, int down, const float* h, int nh, int ns) {
  auto* r = new PortResample;
  r->up = up;
  r->down = down;
  r->h.assign(h, h + nh);
  r->st.assign(ns, 0.0f);
  return r;
}
static void ref_resample_free(void* p) { delete static_cast<PortResample*>(p); }
static long ref_resample_run(void* p, const float* x, long n, float*) {
  auto* r = static_cast<PortResample*>(p);
  r->y.resize(or_resample_len(r->up, r->down, n) + 1);
  return or_resample(r->up, r->down, x, n, r->h.data(), (int)r->h.size(), r->st.data(), (int)r->st.size(),
                     r->y.data());
}
static void* ref_block_new(const float* h, int nh, int ns) {
  auto* r = new PortBlock;
  r->h.assign(h, h + nh);
  r->si.assign(ns, 0.0f);
  r->sq.assign(ns, 0.0f);
  return r;
}
static void ref_block_free(void* p) { delete static_cast<PortBlock*>(p); }
static long ref_block_run(void* p, const float* I, const float* Q, long n, float*, float*) {
  auto* r = static_cast<PortBlock*>(p);
  r->yi.resize(n);
  r->yq.resize(n);
  or_fir_block(I, n, r->h.data(), (int)r->h.size(), r->si.data(), (int)r->si.size(), r->yi.data());
  return or_fir_block(Q, n, r->h.data(), (int)r->h.size(), r->sq.data(), (int)r->sq.size(), r->yq.data());
}
#endif

extern char** environ;

namespace {

using clk = std::chrono::steady_clock;

std::vector<int> affinity_cpus() {
  cpu_set_t set;
  CPU_ZERO(&set);
  std::vector<int> cpus;
  if (sched_getaffinity(0, sizeof set, &set) == 0)
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &set)) cpus.push_back(c);
  if (cpus.empty()) cpus.push_back(0);
  return cpus;
}

// The CPU share this process may use: the affinity set, capped by the
// cgroup CPU quota (a GPU box's container sees every core of the machine in
// its affinity set but is granted a fraction of them) and by
// OMP_NUM_THREADS when the environment sets it to the same share.
struct Share {
  size_t affinity;
  int quota;  // ceil(cgroup quota / period), 0 = unlimited / unknown
  int omp;    // OMP_NUM_THREADS, 0 = unset
  int cores;
};

int read_quota() {
  long q = -1, per = 0;
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2: "<quota|max> <period>"
    char buf[64] = {};
    if (std::fscanf(f, "%63s %ld", buf, &per) == 2 && std::strcmp(buf, "max") != 0) q = std::atol(buf);
    std::fclose(f);
  } else if (FILE* f1 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {  // cgroup v1
    if (std::fscanf(f1, "%ld", &q) != 1) q = -1;
    std::fclose(f1);
    if (FILE* f2 = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (std::fscanf(f2, "%ld", &per) != 1) per = 0;
      std::fclose(f2);
    }
  }
  return (q > 0 && per > 0) ? (int)((q + per - 1) / per) : 0;
}

Share cpu_share() {
  Share s;
  s.affinity = affinity_cpus().size();
  s.quota = read_quota();
  const char* e = std::getenv("OMP_NUM_THREADS");
  s.omp = e ? std::atoi(e) : 0;
  s.cores = (int)s.affinity;
  if (s.quota > 0 && s.quota < s.cores) s.cores = s.quota;
  if (s.omp > 0 && s.omp < s.cores) s.cores = s.omp;
  return s;
}

// Synthetic baseband FM at 2.4 MS/s: message 0.8 sin(2pi 1k t)
// + 0.1 sin(2pi 19k t), 75 kHz deviation, amplitude 0.7, quantised to the
// wire's u8 levels.  `seed` shifts the phase so streams differ.
std::vector<unsigned char> synth_u8(long pairs, unsigned seed) {
  std::vector<unsigned char> iq(2 * pairs);
  const double fs = 2.4e6, kf = 2 * M_PI * 75e3 / fs;
  double phase = 0.37 * seed;
  for (long i = 0; i < pairs; ++i) {
    const double t = (i + 1000.0 * seed) / fs;
    const double m = 0.8 * std::sin(2 * M_PI * 1e3 * t) + 0.1 * std::sin(2 * M_PI * 19e3 * t);
    phase += kf * m;
    const double I = 0.7 * std::cos(phase), Q = 0.7 * std::sin(phase);
    auto q = [](double x) {
      long v = std::lround(128.0 * x + 128.0);
      return (unsigned char)(v < 0 ? 0 : v > 255 ? 255 : v);
    };
    iq[2 * i] = q(I);
    iq[2 * i + 1] = q(Q);
  }
  return iq;
}

enum Kind { kFrontend, kResample, kFir1024 };

int run_kernel(Kind kind, long n, double seconds, int threads) {
  const std::vector<int> cpus = affinity_cpus();
  const Share share = cpu_share();
  if (threads <= 0) threads = share.cores;
  // the taps the bench's config designs (impulseResponseLPF, src/filter.cpp:14-29)
  std::vector<float> h;
  if (kind == kFrontend) {
    h.resize(101);
    ref_taps_lpf(2.4e6f, 100e3f, 101, 1, h.data());
  } else if (kind == kResample) {
    h.resize(151 * 147);
    ref_taps_lpf(240e3f * 147, 16e3f, 151 * 147, 147, h.data());
  } else {
    h.resize(1024);
    ref_taps_lpf(2.4e6f, 100e3f, 1024, 1, h.data());
  }
  // 4 blocks per thread (planar float, the filter.h boundary), as
  // src/iofunc.cpp:113-119 + src/project.cpp:78-81 produce them
  std::vector<std::vector<float>> I(4 * threads), Q(4 * threads);
  for (int b = 0; b < 4 * threads; ++b) {
    const std::vector<unsigned char> iq = synth_u8(n, 1 + b);
    I[b].resize(n);
    Q[b].resize(n);
    for (long i = 0; i < n; ++i) {
      I[b][i] = (float)((iq[2 * i] - 128) / 128.0);
      Q[b][i] = (float)((iq[2 * i + 1] - 128) / 128.0);
    }
  }
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<long long> pairs(threads, 0);
  std::vector<double> secs(threads, 0.0);
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&, t] {
      // pin one thread per core only when the whole affinity set is ours; on
      // a quota-limited share (a GPU box grants 16 of 256) the first cores of
      // the set are not ours alone, and the scheduler places the threads
      if (share.cores == (int)share.affinity && threads <= (int)cpus.size()) {
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(cpus[t % cpus.size()], &one);
        pthread_setaffinity_np(pthread_self(), sizeof one, &one);
      }
      void* f = kind == kFrontend   ? ref_front_new(h.data(), 101, 100)
                : kind == kResample ? ref_resample_new(147, 800, h.data(), (int)h.size(), 150)
                                    : ref_block_new(h.data(), 1024, 1023);
      std::vector<float> demod(n / 10);
      ready.fetch_add(1);
      while (!go.load()) std::this_thread::yield();
      const auto t0 = clk::now();
      long long done = 0;
      int b = 0;
      double el = 0;
      do {
        const float* xi = I[4 * t + b].data();
        const float* xq = Q[4 * t + b].data();
        if (kind == kFrontend)
          ref_front_run(f, 10, xi, xq, n, demod.data());
        else if (kind == kResample)
          ref_resample_run(f, xi, n, nullptr);  // the IF (one channel: the demodulated stream)
        else
          ref_block_run(f, xi, xq, n, nullptr, nullptr);
        done += n;
        b = (b + 1) & 3;
        el = std::chrono::duration<double>(clk::now() - t0).count();
      } while (el < seconds);
      pairs[t] = done;
      secs[t] = el;
      if (kind == kFrontend)
        ref_front_free(f);
      else if (kind == kResample)
        ref_resample_free(f);
      else
        ref_block_free(f);
    });
  }
  while (ready.load() < threads) std::this_thread::yield();
  go.store(true);
  for (auto& th : pool) th.join();
  long long total = 0;
  double wall = 0;
  for (int t = 0; t < threads; ++t) {
    total += pairs[t];
    wall = secs[t] > wall ? secs[t] : wall;
  }
  std::printf("{\"pairs\": %lld, \"seconds\": %.6f, \"threads\": %d, \"affinity\": %zu, \"cgroup_quota\": %d, "
              "\"omp_num_threads\": %d}\n",
              total, wall, threads, share.affinity, share.quota, share.omp);
  return 0;
}

int run_program(const char* prog, long blocks, int procs, const char* channel) {
  const long block_bytes = 1024L * 5 * 10 * 2;  // src/project.cpp:188 (mode 0)
  // 16 distinct blocks, cycled
  const std::vector<unsigned char> pool = synth_u8(16 * block_bytes / 2, 7);
  signal(SIGPIPE, SIG_IGN);
  struct Child {
    pid_t pid = -1;
    int in = -1, out = -1;
    long long pcm = 0;
  };
  std::vector<Child> kids(procs);
  const auto t0 = clk::now();
  for (int p = 0; p < procs; ++p) {
    int pin[2], pout[2];
    // close-on-exec: no child may inherit another child's pipe ends
    if (pipe2(pin, O_CLOEXEC) || pipe2(pout, O_CLOEXEC)) return 2;
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_adddup2(&fa, pin[0], 0);
    posix_spawn_file_actions_adddup2(&fa, pout[1], 1);
    posix_spawn_file_actions_addclose(&fa, pin[1]);
    posix_spawn_file_actions_addclose(&fa, pout[0]);
    // the program's per-block progress lines (src/project.cpp) go nowhere
    posix_spawn_file_actions_addopen(&fa, 2, "/dev/null", O_WRONLY, 0);
    char a0[] = "project", a1[] = "0", a2[16];
    std::snprintf(a2, sizeof a2, "%s", channel);
    char* argv[] = {a0, a1, a2, nullptr};
    if (posix_spawn(&kids[p].pid, prog, &fa, nullptr, argv, environ) != 0) return 3;
    posix_spawn_file_actions_destroy(&fa);
    close(pin[0]);
    close(pout[1]);
    kids[p].in = pin[1];
    kids[p].out = pout[0];
  }
  std::vector<std::thread> io;
  for (int p = 0; p < procs; ++p) {
    io.emplace_back([&, p] {  // feeder
      for (long b = 0; b < blocks; ++b) {
        const unsigned char* src = pool.data() + (b % 16) * block_bytes;
        long off = 0;
        while (off < block_bytes) {
          const ssize_t w = write(kids[p].in, src + off, block_bytes - off);
          if (w <= 0) return;
          off += w;
        }
      }
      close(kids[p].in);
    });
    io.emplace_back([&, p] {  // drain
      std::vector<char> buf(1 << 16);
      for (;;) {
        const ssize_t r = read(kids[p].out, buf.data(), buf.size());
        if (r <= 0) break;
        kids[p].pcm += r;
      }
      close(kids[p].out);
    });
  }
  for (auto& th : io) th.join();
  for (auto& k : kids) {
    int st = 0;
    waitpid(k.pid, &st, 0);
  }
  const double wall = std::chrono::duration<double>(clk::now() - t0).count();
  long long pcm = 0;
  for (auto& k : kids) pcm += k.pcm;
  std::printf("{\"pairs\": %lld, \"seconds\": %.6f, \"procs\": %d, \"pcm_bytes\": %lld}\n",
              (long long)procs * blocks * (block_bytes / 2), wall, procs, pcm);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 2 && !std::strcmp(argv[1], "cores")) {
    std::printf("%d\n", cpu_share().cores);
    return 0;
  }
  if (argc == 5 && (!std::strcmp(argv[1], "frontend") || !std::strcmp(argv[1], "resample") ||
                    !std::strcmp(argv[1], "fir1024"))) {
    const Kind k = !std::strcmp(argv[1], "frontend") ? kFrontend : !std::strcmp(argv[1], "resample") ? kResample
                                                                                                      : kFir1024;
    return run_kernel(k, std::atol(argv[2]), std::atof(argv[3]), std::atoi(argv[4]));
  }
  if ((argc == 5 || argc == 6) && !std::strcmp(argv[1], "program")) {
    int procs = std::atoi(argv[4]);
    if (procs <= 0) procs = cpu_share().cores;
    const char* ch = argc == 6 ? argv[5] : "mono";
    if (std::strcmp(ch, "mono") && std::strcmp(ch, "stereo")) return 2;
    return run_program(argv[2], std::atol(argv[3]), procs, ch);
  }
  std::fprintf(stderr,
               "usage: cpu_bench frontend|resample|fir1024 <block> <seconds> <threads|0>\n"
               "       cpu_bench program <project_binary> <blocks> <procs|0> [mono|stereo]\n"
               "       cpu_bench cores\n");
  return 2;
}

// sdr_project.cpp -- the reference's `project` program (src/project.cpp) with
// its block loop re-done for the GPU.
//
// Same command line, same stdin (u8 IQ), same stdout (s16 PCM, mono or
// interleaved L/R), same stderr lines, same exit status.  What changes is
// how a block moves:
//   reference: per block, spawn a front-end thread and a back-end thread
//              that meet in a threadSafeQ (src/project.cpp:292-305,
//              src/threadSafeQ.cpp), every stage on the CPU;
//   here:      the whole block -- front end, mono path, stereo path, s16
//              output stage -- is one stream-ordered device call
//              (sdr_mono_pcm_u8_dev / sdr_stereo_pcm_u8_dev).  Two pinned
//              input and two pinned output buffers form a ring: while the
//              device works on block b (H2D, kernels, D2H), the host reads
//              block b+1 from stdin and writes block b-1's PCM to stdout.
// Filter state never leaves the device.  Output bytes equal the reference's
// (tests/test_dropin.py).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "sdr_hip.h"

namespace {

sdr_ctx* g_ctx = nullptr;

void check(int rc, const char* what) {
  if (rc != SDR_OK) {
    std::fprintf(stderr, "sdr_project: %s: %s (%s)\n", what, sdr_strerror(rc),
                 g_ctx ? sdr_ctx_last_error(g_ctx) : "");
    std::exit(2);
  }
}

void* dev_zeros(size_t bytes) {
  void* p = nullptr;
  check(sdr_dev_alloc(g_ctx, bytes, &p), "dev_alloc");
  check(sdr_dev_memset(g_ctx, p, 0, bytes), "dev_memset");
  return p;
}

const float* dev_copy(const std::vector<float>& v) {
  void* p = nullptr;
  check(sdr_dev_alloc(g_ctx, v.size() * sizeof(float), &p), "dev_alloc");
  check(sdr_copy_h2d(g_ctx, p, v.data(), v.size() * sizeof(float)), "copy_h2d");
  return static_cast<const float*>(p);
}

std::vector<float> lpf(float Fs, float Fc, int ntaps, int up) {
  std::vector<float> h(ntaps);
  check(sdr_taps_lpf(Fs, Fc, ntaps, up, h.data()), "taps_lpf");
  return h;
}

std::vector<float> bpf(float Fs, float Fb, float Fe, int ntaps) {
  std::vector<float> h(ntaps);
  check(sdr_taps_bpf(Fs, Fb, Fe, ntaps, 1, h.data()), "taps_bpf");
  return h;
}

// fread until n bytes or end of input; the reference's std::cin.read
size_t read_full(uint8_t* dst, size_t n) {
  size_t got = 0;
  while (got < n) {
    const size_t r = std::fread(dst + got, 1, n - got, stdin);
    if (r == 0) break;
    got += r;
  }
  return got;
}

}  // namespace

int main(int argc, char* argv[]) {
  // src/project.cpp:155-176: argument handling and messages
  int mode = 0;
  bool mono = true;
  if (argc == 3) {
    mode = std::atoi(argv[1]);
    const std::string channel = argv[2];
    mono = channel == "stereo" ? false : true;
    if (mode > 3) {
      std::cerr << "Wrong mode: " << mode << std::endl;
      std::exit(1);
    } else if (channel != "mono" && channel != "stereo") {
      std::cerr << "Wrong parameter: " << channel << ", must be mono or stereo" << std::endl;
    }
  } else {
    std::cerr << "Usage: " << argv[0] << std::endl;
    std::cerr << "or " << std::endl;
    std::cerr << "Usage: " << argv[0] << " <mode>" << std::endl;
    std::cerr << "or " << std::endl;
    std::cerr << "Usage: " << argv[0] << " <mode> <mono/stereo>" << std::endl;
    std::cerr << "\t\t <mode> is a value from 0 to 3" << std::endl;
    std::exit(1);
  }
  std::cerr << "Operating in mode " << mode << (mono ? " mono" : " stereo") << std::endl;

  // src/project.cpp:178-238: the mode table (negative modes take the default row)
  const int num_taps = 101;
  float rf_Fs = 2.4e6f, audio_Fs = 240e3f;
  int rf_decim = 10, audio_decim = 5, audio_up = 1, block_size = 1024 * 5 * 10 * 2;
  switch (mode) {
    case 1:
      rf_Fs = 1.44e6f, rf_decim = 5, audio_Fs = 288e3f, audio_decim = 8, audio_up = 1;
      block_size = 1024 * audio_decim * rf_decim * 2;
      break;
    case 2:
      rf_Fs = 2.4e6f, rf_decim = 10, audio_Fs = 240e3f, audio_decim = 800, audio_up = 147;
      block_size = 10 * audio_decim * rf_decim * 2;
      break;
    case 3:
      rf_Fs = 1.92e6f, rf_decim = 5, audio_Fs = 384e3f, audio_decim = 1280, audio_up = 147;
      block_size = 10 * audio_decim * rf_decim * 2;
      break;
    default:
      break;
  }
  const int audio_taps = num_taps * audio_up;
  const long long npairs = block_size / 2;
  const long long nd = npairs / rf_decim;
  const long long na = sdr_resample_out_len(audio_up, audio_decim, nd);
  const long long pcm_len = na * (mono ? 1 : 2);

  const char* devenv = std::getenv("SDR_DEVICE");
  check(sdr_ctx_create(devenv ? std::atoi(devenv) : 0, &g_ctx), "ctx_create");

  // src/project.cpp:258-273: coefficients (host design, bit-identical), on the device
  sdr_stereo_taps taps;
  taps.h_rf = dev_copy(lpf(rf_Fs, 100e3f, num_taps, 1));
  taps.rf_taps = num_taps;
  taps.h_audio = dev_copy(lpf(audio_Fs * (float)audio_up, 16e3f, audio_taps, audio_up));
  taps.audio_taps = audio_taps;
  taps.h_pilot = dev_copy(bpf(audio_Fs, 18.5e3f, 19.5e3f, num_taps));
  taps.h_stereo = dev_copy(bpf(audio_Fs, 22e3f, 54e3f, num_taps));
  taps.bpf_taps = num_taps;

  // src/project.cpp:243-257 + 25-55: state, zero except the PLL's 1, 0, 0, 0, 0, 1
  sdr_stereo_state st;
  st.ns_rf = num_taps - 1;
  st.state_i = static_cast<float*>(dev_zeros(st.ns_rf * sizeof(float)));
  st.state_q = static_cast<float*>(dev_zeros(st.ns_rf * sizeof(float)));
  st.prev_i = static_cast<float*>(dev_zeros(sizeof(float)));
  st.prev_q = static_cast<float*>(dev_zeros(sizeof(float)));
  st.ns_delay = num_taps / 2;
  st.delay_state = static_cast<float*>(dev_zeros(st.ns_delay * sizeof(float)));
  st.ns_audio = num_taps - 1;
  st.state_audio = static_cast<float*>(dev_zeros(st.ns_audio * sizeof(float)));
  st.stereo_lp_state = static_cast<float*>(dev_zeros(st.ns_audio * sizeof(float)));
  st.ns_bpf = num_taps - 1;
  st.pilot_state = static_cast<float*>(dev_zeros(st.ns_bpf * sizeof(float)));
  st.stereo_state = static_cast<float*>(dev_zeros(st.ns_bpf * sizeof(float)));
  const float pll0[6] = {1.0f, 0.0f, 0.0f, 0.0f, 0.0f, 1.0f};
  void* pll = nullptr;
  check(sdr_dev_alloc(g_ctx, sizeof pll0, &pll), "dev_alloc");
  check(sdr_copy_h2d(g_ctx, pll, pll0, sizeof pll0), "copy_h2d");
  st.pll = static_cast<float*>(pll);

  // the ring: 2 pinned inputs, 2 pinned outputs, 2 device input/output pairs
  uint8_t* h_in[2];
  int16_t* h_out[2];
  void* d_in[2];
  void* d_out[2];
  sdr_event* done[2];
  for (int i = 0; i < 2; ++i) {
    check(sdr_host_alloc(g_ctx, block_size, reinterpret_cast<void**>(&h_in[i])), "host_alloc");
    check(sdr_host_alloc(g_ctx, pcm_len * sizeof(int16_t), reinterpret_cast<void**>(&h_out[i])), "host_alloc");
    check(sdr_dev_alloc(g_ctx, block_size, &d_in[i]), "dev_alloc");
    check(sdr_dev_alloc(g_ctx, pcm_len * sizeof(int16_t), &d_out[i]), "dev_alloc");
    check(sdr_event_create(g_ctx, &done[i]), "event_create");
  }

  // One block's device work: copy in, the whole mono/stereo path, copy out
  // (~10 launches).  For one stream these are latency-bound, so after the
  // first block each ring slot's sequence is captured once into a HIP graph
  // and replayed: one launch per block (SDR_PROJECT_NO_GRAPH=1 launches them
  // one by one).
  auto enqueue = [&](int k) {
    check(sdr_copy_h2d_async(g_ctx, d_in[k], h_in[k], block_size), "copy_h2d_async");
    const uint8_t* iq = static_cast<const uint8_t*>(d_in[k]);
    int16_t* pcm = static_cast<int16_t*>(d_out[k]);
    if (mono)
      check(sdr_mono_pcm_u8_dev(g_ctx, rf_decim, iq, npairs, 1, 2 * npairs, taps.h_rf, num_taps, st.state_i,
                                st.state_q, st.ns_rf, st.prev_i, st.prev_q, st.delay_state, st.ns_delay, audio_up,
                                audio_decim, taps.h_audio, audio_taps, st.state_audio, st.ns_audio, pcm, pcm_len),
            "mono_pcm_u8_dev");
    else
      check(sdr_stereo_pcm_u8_dev(g_ctx, rf_decim, iq, npairs, 1, 2 * npairs, audio_up, audio_decim, audio_Fs, &taps,
                                  &st, pcm, pcm_len),
            "stereo_pcm_u8_dev");
    check(sdr_copy_d2h_async(g_ctx, h_out[k], d_out[k], pcm_len * sizeof(int16_t)), "copy_d2h_async");
  };
  const char* nog = std::getenv("SDR_PROJECT_NO_GRAPH");
  const bool use_graph = !(nog && std::atoi(nog) != 0);
  sdr_graph* graph[2] = {nullptr, nullptr};

  // Stereo: the block is cut where the PLL recurrence starts (sdr_stereo_front_u8_dev /
  // sdr_stereo_back_dev, disjoint state).  The front stage runs on g_ctx's stream, the
  // back stage on a second context's, so block b+1's copy-in, front end and band-pass
  // filters overlap block b's recurrence -- the one-lane PLL is most of a stereo block
  // (DESIGN.md 4.7).  Each ring slot has its own work object; front(b) waits for
  // back(b-2) (the slot's previous user), back(b) for front(b).  SDR_PROJECT_SPLIT=0
  // runs the whole block as one call instead.
  // SDR_PROJECT_SPLIT=2 (the default) keeps the second stream on the recurrences alone:
  // block b's post stage (NCO, stereo resampler, PCM, copy-out) runs on g_ctx's stream
  // after block b+1's front stage, once recurrence b is done (sdr_stereo_pll_dev /
  // sdr_stereo_post_dev; bench.py --stereo-pipeline 2).  Its PCM then leaves one block
  // later than under SPLIT=1, which is when the loop below writes it out anyway.
  const char* spl = std::getenv("SDR_PROJECT_SPLIT");
  // mode-0 stereo, 3,000 blocks: 3.358 s split vs 3.560 s one call (profiles/r04e/ab.txt)
  const int split_mode = mono ? 0 : (spl ? std::atoi(spl) : 2);
  const bool split = split_mode != 0;
  const bool post_front = split_mode == 2;
  sdr_ctx* g_back = nullptr;
  sdr_stereo_work* work[2] = {nullptr, nullptr};
  sdr_event* front_done[2] = {nullptr, nullptr};
  sdr_event* pll_done[2] = {nullptr, nullptr};
  sdr_graph* graph_back[2] = {nullptr, nullptr};
  sdr_graph* graph_post[2] = {nullptr, nullptr};
  if (split) {
    check(sdr_ctx_create(devenv ? std::atoi(devenv) : 0, &g_back), "ctx_create");
    for (int i = 0; i < 2; ++i) {
      check(sdr_stereo_work_create(g_ctx, rf_decim, npairs, audio_up, audio_decim, 1, &work[i]), "stereo_work_create");
      check(sdr_event_create(g_ctx, &front_done[i]), "event_create");
      check(sdr_event_create(g_ctx, &pll_done[i]), "event_create");
    }
  }
  auto enqueue_front = [&](int k) {
    check(sdr_copy_h2d_async(g_ctx, d_in[k], h_in[k], block_size), "copy_h2d_async");
    check(sdr_stereo_front_u8_dev(g_ctx, static_cast<const uint8_t*>(d_in[k]), 2 * npairs, &taps, &st, work[k]),
          "stereo_front_u8_dev");
  };
  auto enqueue_back = [&](int k) {
    if (post_front) {
      check(sdr_stereo_pll_dev(g_back, audio_Fs, &st, work[k]), "stereo_pll_dev");
      return;
    }
    check(sdr_stereo_back_dev(g_back, audio_Fs, &taps, &st, work[k], static_cast<int16_t*>(d_out[k]), pcm_len),
          "stereo_back_dev");
    check(sdr_copy_d2h_async(g_back, h_out[k], d_out[k], pcm_len * sizeof(int16_t)), "copy_d2h_async");
  };
  auto enqueue_post = [&](int k) {  // SPLIT=2: on g_ctx, after recurrence k
    check(sdr_stereo_post_dev(g_ctx, &taps, &st, work[k], static_cast<int16_t*>(d_out[k]), pcm_len),
          "stereo_post_dev");
    check(sdr_copy_d2h_async(g_ctx, h_out[k], d_out[k], pcm_len * sizeof(int16_t)), "copy_d2h_async");
  };
  // run f on ctx directly (block 0 sizes the scratch) or as slot k's recorded graph
  auto run = [&](sdr_ctx* ctx, sdr_graph** g, bool direct, auto&& f) {
    if (direct) {
      f();
      return;
    }
    if (!*g) {
      check(sdr_graph_begin(ctx), "graph_begin");
      f();
      check(sdr_graph_end(ctx, g), "graph_end");
    }
    check(sdr_graph_launch(ctx, *g), "graph_launch");
  };

  auto flush = [&](unsigned b) {  // wait for block b and write its PCM (src/project.cpp:315)
    check(sdr_event_synchronize(g_ctx, done[b & 1]), "event_synchronize");
    std::fwrite(h_out[b & 1], sizeof(int16_t), pcm_len, stdout);
  };

  // SPLIT=2: block b's post stage, after its recurrence (the first one sizes its scratch)
  auto post = [&](unsigned b) {
    const int j = b & 1;
    check(sdr_ctx_wait_event(g_ctx, pll_done[j]), "wait_event");
    run(g_ctx, &graph_post[j], b == 0 || !use_graph, [&] { enqueue_post(j); });
    check(sdr_event_record(g_ctx, done[j]), "event_record");
  };

  for (unsigned int block_id = 0;; block_id++) {
    std::cerr << "Block number " << block_id << std::endl;
    const int k = block_id & 1;
    // h_in[k] was last used by block_id - 2, whose copy finished before flush(block_id - 2)
    if (read_full(h_in[k], block_size) != (size_t)block_size) {
      if (post_front && block_id > 0) post(block_id - 1);
      if (block_id > 0) flush(block_id - 1);
      std::fflush(stdout);
      std::cerr << "End of input stream reached" << std::endl;
      std::exit(1);  // as the reference (src/project.cpp:294-297)
    }
    // the first block sizes the library's scratch (no allocation may happen
    // inside a capture); then each ring slot's sequence is recorded once and replayed
    const bool direct = block_id == 0 || !use_graph;
    if (split) {
      // back(b-2) released work[k] (SPLIT=2: post(b-2), earlier on this stream)
      if (block_id >= 2 && !post_front) check(sdr_ctx_wait_event(g_ctx, done[k]), "wait_event");
      run(g_ctx, &graph[k], direct, [&] { enqueue_front(k); });
      check(sdr_event_record(g_ctx, front_done[k]), "event_record");
      check(sdr_ctx_wait_event(g_back, front_done[k]), "wait_event");
      run(g_back, &graph_back[k], direct, [&] { enqueue_back(k); });
      check(sdr_event_record(g_back, post_front ? pll_done[k] : done[k]), "event_record");
      if (post_front && block_id > 0) post(block_id - 1);
    } else {
      run(g_ctx, &graph[k], direct, [&] { enqueue(k); });
      check(sdr_event_record(g_ctx, done[k]), "event_record");
    }
    // block_id - 1's PCM goes out while the device runs block_id and the
    // next read waits on stdin
    if (block_id > 0) flush(block_id - 1);
  }
}

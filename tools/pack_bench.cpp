// Host budget of the generic-batch pipeline: how many CPU
// threads one process needs to feed N GPUs through cordahip_sig_verify.
//
// Per lane the host does what host_batch.cpp's sig_pipeline does on its pool,
// with the same code (corda_amd/csrc/pack_rows.hpp): classify the lane (scheme,
// key length, message length), pack its row into the stage's (here: ordinary)
// buffers -- Ed25519: key 32 + signature 64 + message 32 B + pre-status;
// ECDSA: SEC1 key in a 65-byte slot, DER signature in a 72-byte slot, lengths,
// CSR message -- and, when the GPU is done, scatter its status back to the
// caller's array and build the verdict words. Batches are CSR arrays as the JVM
// hands them over (random bytes of the right lengths: the work does not depend
// on the values). Output: one JSON line per (scheme, threads) with lanes/s.
// Built and run by tests/test_pack_bench.py (g++, no GPU).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <pthread.h>
#include <sched.h>

#include <thread>
#include <vector>

#include "../corda_amd/csrc/numa_place.hpp"
#include "../corda_amd/csrc/pack_rows.hpp"

using namespace cordahip::rt;

namespace {

struct View {  // runtime.hpp MsgView without the device part
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* tx_of = nullptr;
  const uint8_t* ptr(uint64_t i) const { return base + off[i]; }
  uint64_t len(uint64_t i) const { return off[i + 1] - off[i]; }
};

struct Batch {
  std::vector<uint8_t> scheme, key, sig, msg, status;
  std::vector<uint64_t> key_off, sig_off, msg_off, verdict;
  cordahip_sig_batch b{};
};

void make(Batch& B, uint64_t n, bool ecdsa) {
  std::mt19937_64 g(7);
  B.scheme.resize(n);
  B.key_off.resize(n + 1);
  B.sig_off.resize(n + 1);
  B.msg_off.resize(n + 1);
  uint64_t ko = 0, so = 0, mo = 0;
  for (uint64_t i = 0; i < n; i++) {
    B.scheme[i] = ecdsa ? (uint8_t)(2 + (i & 1)) : (uint8_t)CORDAHIP_SCHEME_EDDSA_ED25519_SHA512;
    B.key_off[i] = ko, B.sig_off[i] = so, B.msg_off[i] = mo;
    ko += ecdsa ? 65 : 32;
    so += ecdsa ? 70 + (i % 3) : 64;
    mo += 32;
  }
  B.key_off[n] = ko, B.sig_off[n] = so, B.msg_off[n] = mo;
  auto fill = [&](std::vector<uint8_t>& v, uint64_t m) {
    v.resize(m);
    for (uint64_t i = 0; i < m; i += 8) {
      const uint64_t x = g();
      std::memcpy(&v[i], &x, std::min<uint64_t>(8, m - i));
    }
  };
  fill(B.key, ko);
  fill(B.sig, so);
  fill(B.msg, mo);
  B.status.assign(n, 0);
  B.verdict.assign((n + 63) / 64, 0);
  B.b = cordahip_sig_batch{n, B.scheme.data(), B.key.data(), B.key_off.data(), B.sig.data(), B.sig_off.data(),
                           B.msg.data(), B.msg_off.data(), B.status.data(), B.verdict.data(), 0u,
                           (uint64_t)B.key.size(), (uint64_t)B.sig.size(), (uint64_t)B.msg.size()};
}

// lanes [lo, hi) through classify, pack, scatter, verdict words (the per-lane host work of a chunk)
void work(const Batch& B, bool ecdsa, uint64_t lo, uint64_t hi, std::vector<uint8_t>& rows, std::vector<uint64_t>& mo_v,
          std::vector<uint16_t>& cls) {
  const cordahip_sig_batch* b = &B.b;
  const View mv{B.msg.data(), B.msg_off.data()};
  const uint64_t m = hi - lo;
  cls.resize(m);
  for (uint64_t r = 0; r < m; r++) {
    uint64_t ml;
    cls[r] = classify(b, mv, lo + r, ml);
  }
  if (!ecdsa) {
    rows.resize(m * 130);
    uint8_t *k = rows.data(), *s = k + m * 32, *msg = s + m * 64, *pre = msg + m * 32;
    for (uint64_t r = 0; r < m; r++) pack_ed_row(b, mv, true, lo + r, 32, k + r * 32, s + r * 64, msg + r * 32, pre + r);
  } else {
    rows.resize(m * (1 + 65 + 1 + 72 + 1 + 32 + 1));
    mo_v.resize(m);
    uint8_t *sc = rows.data(), *k = sc + m, *kl = k + m * 65, *sg = kl + m, *sl = sg + m * 72, *msg = sl + m,
            *pre = msg + m * 32;
    uint64_t mo = 0;
    for (uint64_t r = 0; r < m; r++)
      pack_ec_row(b, mv, true, lo + r, r, sc, k, kl, sg, sl, msg, mo_v.data(), pre, mo, nullptr);
  }
  // the GPU's statuses back to the caller's lanes, then the verdict words (64-aligned ranges)
  const uint8_t* st = rows.data();
  for (uint64_t r = 0; r < m; r++) B.b.status[lo + r] = st[r] & 1;
  for (uint64_t w = lo / 64; w < (hi + 63) / 64; w++) {
    uint64_t v = 0;
    for (uint64_t j = 0; j < 64 && w * 64 + j < B.b.n; j++) v |= (uint64_t)(B.b.status[w * 64 + j] == 0) << j;
    B.b.verdict[w] = v;
  }
}

}  // namespace

// POOLS > 0: one pool per simulated device, as the library runs them (numa_place.hpp):
// the allowed CPUs grouped by NUMA node, the pools spread over the nodes and each
// bound to a disjoint slice of its node's CPUs; every pool first-touches its own
// batch (a device's shard) from a bound thread, then all pools pack at once. Prints
// the aggregate and the slowest pool's lanes/s per scheme.
int pools_mode(uint64_t n, int threads, int pools) {
  std::vector<int> allowed;
  {
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0)
      for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &cs)) allowed.push_back(c);
  }
  std::vector<std::vector<int>> by_node;  // allowed CPUs of each node that has any
  for (int node = 0; node < 64; node++) {
    std::string t;
    if (!cordahip::rt::read_text("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", t)) continue;
    std::vector<int> c = cordahip::rt::parse_cpulist(t), mine;
    std::set_intersection(c.begin(), c.end(), allowed.begin(), allowed.end(), std::back_inserter(mine));
    if (!mine.empty()) by_node.push_back(mine);
  }
  if (by_node.empty()) by_node.push_back(allowed);
  std::vector<std::vector<int>> slice(pools);
  for (int k = 0; k < pools; k++) {  // pool k on node k * nodes / pools, the node's pools split its CPUs
    const int nn = (int)by_node.size(), node = k * nn / pools;
    int first = 0, count = 0;
    for (int j = 0; j < pools; j++)
      if (j * nn / pools == node) {
        if (j < k) first++;
        count++;
      }
    const auto& c = by_node[node];
    size_t lo = c.size() * first / count, hi = c.size() * (first + 1) / count;
    if (hi <= lo) {  // more pools than CPUs on the node: one CPU each, shared
      hi = std::min(c.size(), lo + 1);
      lo = hi - 1;
    }
    slice[k].assign(c.begin() + (long)lo, c.begin() + (long)hi);
  }
  const int per = std::max(1, threads / pools);
  auto bind = [](const std::vector<int>& cpus) {
    cpu_set_t cs;
    CPU_ZERO(&cs);
    for (int c : cpus) CPU_SET(c, &cs);
    (void)pthread_setaffinity_np(pthread_self(), sizeof(cs), &cs);
  };
  for (int ec = 0; ec < 2; ec++) {
    std::vector<Batch> B(pools);
    {
      std::vector<std::thread> th;
      for (int k = 0; k < pools; k++) th.emplace_back([&, k] { bind(slice[k]); make(B[k], n, ec); });
      for (auto& x : th) x.join();
    }
    double best_all = 1e30;
    // each thread's staging rows persist across the repetitions (the library's pinned
    // stages do across chunks): the first repetition pays their first touch, best of 4
    std::vector<std::vector<uint8_t>> rows(pools * per);
    std::vector<std::vector<uint64_t>> mo(pools * per);
    std::vector<std::vector<uint16_t>> cls(pools * per);
    for (int rep = 0; rep < 4; rep++) {
      const auto t0 = std::chrono::steady_clock::now();
      std::vector<std::thread> th;
      for (int k = 0; k < pools; k++)
        for (int q = 0; q < per; q++)
          th.emplace_back([&, k, q] {
            bind(slice[k]);
            const uint64_t step = (n / per + 63) / 64 * 64, lo = std::min<uint64_t>(n, q * step),
                           hi = std::min<uint64_t>(n, lo + step);
            work(B[k], ec, lo, hi, rows[k * per + q], mo[k * per + q], cls[k * per + q]);
          });
      for (auto& x : th) x.join();
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (dt < best_all) best_all = dt;
    }
    std::string cpus;
    for (int k = 0; k < pools; k++) cpus += std::string(k ? "; " : "") + std::to_string(slice[k].size());
    printf("{\"scheme\": \"%s\", \"pools\": %d, \"threads_per_pool\": %d, \"lanes_per_pool\": %llu, "
           "\"numa_nodes\": %zu, \"cpus_per_pool\": \"%s\", \"s\": %.4f, \"lanes_per_s\": %.4g, "
           "\"lanes_per_s_per_pool\": %.4g}\n",
           ec ? "ecdsa" : "ed25519", pools, per, (unsigned long long)n, by_node.size(), cpus.c_str(), best_all,
           pools * n / best_all, n / best_all);
    fflush(stdout);
  }
  return 0;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 22);
  const int maxt = argc > 2 ? atoi(argv[2]) : (int)std::thread::hardware_concurrency();
  if (argc > 3 && atoi(argv[3]) > 0) return pools_mode(n, maxt, atoi(argv[3]));
  for (int ec = 0; ec < 2; ec++) {
    Batch B;
    make(B, n, ec);
    std::vector<int> ts{1};
    for (int t = 2; t <= maxt; t *= 2) ts.push_back(t);
    if (ts.back() != maxt && maxt > 1) ts.push_back(maxt);
    for (int t : ts) {
      std::vector<std::vector<uint8_t>> rows(t);
      std::vector<std::vector<uint64_t>> mo(t);
      std::vector<std::vector<uint16_t>> cls(t);
      double best = 1e30;
      for (int rep = 0; rep < 3; rep++) {
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int k = 0; k < t; k++) {
          const uint64_t per = (n / t + 63) / 64 * 64, lo = std::min<uint64_t>(n, k * per),
                         hi = std::min<uint64_t>(n, lo + per);
          th.emplace_back([&, k, lo, hi] { work(B, ec, lo, hi, rows[k], mo[k], cls[k]); });
        }
        for (auto& x : th) x.join();
        best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
      }
      printf("{\"scheme\": \"%s\", \"lanes\": %llu, \"threads\": %d, \"s\": %.4f, \"lanes_per_s\": %.4g, "
             "\"lanes_per_s_per_thread\": %.4g}\n",
             ec ? "ecdsa" : "ed25519", (unsigned long long)n, t, best, n / best, n / best / t);
      fflush(stdout);
    }
  }
  return 0;
}

// Where the Ed25519 ladder's L2 misses are served: Infinity Cache (MALL) or HBM.
//
// rocprofv3 on gfx950 has no MALL counter (the 4,012-counter list of the box,
// profiles/r04_counters_list.txt: TCC_EA0_RDREQ / _DRAM count every L2->fabric
// read, MALL hits included), so the split of the ladder's measured 17.0 KB of
// L2-miss reads per verification (FETCH_SIZE, x2 gfx950 correction) comes from
// this trace-driven model of the kernel's own access stream, CALIBRATED on that
// counter: the model's L2-miss bytes must reproduce the measured FETCH before
// its MALL-miss (= HBM) bytes are believed.
//
// Access stream (ed25519_ladder.hip, ed25519_ws.hpp): lane l's 3,200-B record
// at l * 3200; per window (33 of 4 bits over |c0|, c1 ~ 2^128), one 160-B
// entry of the lane's [1..8](-A) table and one of its [1..8](-R) table
// (192-B stride, sector-aligned), entry |d| - 1 for Booth digit d, digit 0 the
// shared identity entry; every 4th window one 128-B niels entry of each 4.2 MB
// fixed-base table ([k]B, [k]B', 16-bit Booth digits); the record's scalars
// once. Blocks of 256 lanes, dealt round-robin to the 8 XCDs; 512 blocks
// resident (2 waves per SIMD, 247 VGPRs); each XCD's L2 is 4 MB, the MALL
// 256 MB shared; 128-B lines, LRU, the MALL allocating on every L2 miss.
// Two schedules bracket reality: lockstep rounds (every resident block at the
// same window) and staggered (resident blocks at uniformly spread windows).
//
// build: g++ -O2 -std=c++17 -o /tmp/mall_sim tools/mall_sim.cpp; run: /tmp/mall_sim
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <list>
#include <random>
#include <unordered_map>
#include <vector>

struct Lru {
  size_t cap;
  std::list<uint64_t> order;  // front = most recent
  std::unordered_map<uint64_t, std::list<uint64_t>::iterator> where;
  explicit Lru(size_t c) : cap(c) { where.reserve(c * 2); }
  bool touch(uint64_t line) {  // true on hit
    auto it = where.find(line);
    if (it != where.end()) {
      order.splice(order.begin(), order, it->second);
      return true;
    }
    order.push_front(line);
    where[line] = order.begin();
    if (order.size() > cap) {
      where.erase(order.back());
      order.pop_back();
    }
    return false;
  }
};

struct Stats {
  uint64_t lanes = 0, l2_miss = 0, mall_miss = 0, accesses = 0;
};

constexpr uint64_t kLine = 128, kRec = 3200, kEntry = 192, kEntryRead = 160;
constexpr int kWindows = 33, kLanesPerBlock = 256, kXcd = 8, kResident = 512;
constexpr uint64_t kBTab = 1ull << 40, kBEntries = 32769, kIdentity = 1ull << 41;

int booth4(std::mt19937_64& g) {  // |d| of a 4-bit Booth digit: 0 and 8 at 1/16, 1..7 at 1/8
  const int r = (int)(g() & 15);
  return r == 0 ? 0 : r == 15 ? 8 : (r + 1) / 2;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 4;
  for (int staggered = 0; staggered < 2; staggered++) {
    std::mt19937_64 g(7);
    std::vector<Lru> l2(kXcd, Lru(4u << 20 >> 7));
    Lru mall(256u << 20 >> 7);
    Stats st;
    const uint64_t total_blocks = (uint64_t)kResident * rounds;
    // slot state: block id, its window, its lanes' digits
    struct Slot {
      uint64_t block = 0;
      int window = 0;
      Stats acc;  // this block's counts, added to st when it completes
    };
    std::vector<Slot> slot(kResident);
    uint64_t next_block = 0;
    for (int s = 0; s < kResident; s++) {
      slot[s].block = next_block++;
      slot[s].window = staggered ? (int)(g() % kWindows) : 0;
    }
    auto access = [&](Stats& a, int xcd, uint64_t addr, uint64_t bytes) {
      for (uint64_t ln = addr / kLine; ln <= (addr + bytes - 1) / kLine; ln++) {
        a.accesses++;
        if (l2[xcd].touch(ln)) continue;
        a.l2_miss++;
        if (!mall.touch(ln)) a.mall_miss++;
      }
    };
    uint64_t done = 0;
    std::vector<int> order(kResident);
    for (int i = 0; i < kResident; i++) order[i] = i;
    while (done < total_blocks) {
      std::shuffle(order.begin(), order.end(), g);
      for (int s : order) {
        Slot& sl = slot[s];
        const int xcd = (int)(sl.block % kXcd);
        for (int t = 0; t < kLanesPerBlock; t++) {
          const uint64_t lane = sl.block * kLanesPerBlock + t;
          const uint64_t rec = lane * kRec;
          if (sl.window == 0) access(sl.acc, xcd, rec + 16 * kEntry, 128);  // scalars
          const int da = booth4(g), dr = booth4(g);
          access(sl.acc, xcd, da ? rec + (da - 1) * kEntry : kIdentity, kEntryRead);
          access(sl.acc, xcd, dr ? rec + 8 * kEntry + (dr - 1) * kEntry : kIdentity, kEntryRead);
          if (sl.window % 4 == 3) {
            access(sl.acc, xcd, kBTab + (g() % kBEntries) * kLine, kLine);
            access(sl.acc, xcd, kBTab + (kBEntries + g() % kBEntries) * kLine, kLine);
          }
        }
        if (++sl.window == kWindows) {
          // the first generation (cold caches; staggered: partial blocks) is not counted
          if (sl.block >= (uint64_t)kResident) {
            st.lanes += kLanesPerBlock;
            st.accesses += sl.acc.accesses;
            st.l2_miss += sl.acc.l2_miss;
            st.mall_miss += sl.acc.mall_miss;
          }
          done++;
          sl.acc = Stats();
          sl.block = next_block++;
          sl.window = 0;
        }
      }
    }
    const double per = 1.0 / (double)st.lanes;
    printf("{\"schedule\": \"%s\", \"lanes\": %llu, \"l2_miss_bytes_per_lane\": %.0f, "
           "\"hbm_bytes_per_lane\": %.0f, \"mall_hit_bytes_per_lane\": %.0f, \"accessed_bytes_per_lane\": %.0f}\n",
           staggered ? "staggered" : "lockstep", (unsigned long long)st.lanes, st.l2_miss * kLine * per,
           st.mall_miss * kLine * per, (st.l2_miss - st.mall_miss) * kLine * per, st.accesses * kLine * per);
    fflush(stdout);
  }
  return 0;
}

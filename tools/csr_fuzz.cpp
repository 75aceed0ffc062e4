// Mutation fuzzer of the C-ABI's CSR validation (corda_amd/csrc/csr_check.hpp)
// and of the generic batch's per-lane classification and row packing
// (corda_amd/csrc/pack_rows.hpp), on the host, built by tests/test_csr_fuzz.py
// with g++ -fsanitize=address,undefined. The batches come from the JVM, so every
// offset and declared length is untrusted: a bad one must fail the batch with
// CORDAHIP_ERR_INVALID_ARG, never make the host read outside a caller buffer.
//
// Every array lives in a heap block of exactly the entries its declared count
// implies ([n + 1] offsets, blobs of exactly their declared bytes), so a read
// past one is an ASan report. Per round, one batch of each kind is built valid,
// then (most rounds) mutated -- an offset set to 0, to its neighbour +- 1..5, to
// the declared length (+1), to 2^64 - 1 or to a random value; two neighbours
// swapped; a declared length or count lowered --, and:
//   * a generic signature batch (cordahip_sig_batch) runs through the pipeline's
//     order of work: chunks of 1..64 lanes, each classified lane by lane, and
//     packed (Ed25519 rows, ECDSA slots) only when no lane of the chunk is
//     kBadCsr -- the batch is invalid exactly when some lane's ranges are;
//   * transaction batches (txid + signature levels, components, filtered
//     transactions) go through check_txid_batch / check_sig_level /
//     check_txcomp_batch / check_filtered_batch, whose verdict must equal the
//     contract's ground truth; a batch they accept is then walked the way the
//     library walks it (every leaf, signature, item and token range read).
// Exit 0 when every verdict matches; a sanitizer report aborts the process.
//
// usage: csr_fuzz ROUNDS RNG_SEED   (prints one JSON line of counts)
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "../corda_amd/csrc/csr_check.hpp"
#include "../corda_amd/csrc/pack_rows.hpp"

using namespace cordahip::rt;

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {  // splitmix64
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
  }
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
  bool chance(uint64_t pct) { return below(100) < pct; }
};

// an exact-size heap array (an empty one still has a distinct, unreadable address)
template <class T>
struct Arr {
  std::unique_ptr<T[]> p;
  uint64_t n = 0;
  void make(uint64_t k) {
    n = k;
    p.reset(new T[k ? k : 1]);
    if (k) std::memset(p.get(), 0, sizeof(T) * k);
  }
  T* get() const { return n ? p.get() : nullptr; }
};

struct SerialPar {
  template <class F>
  void operator()(uint64_t n, uint64_t, F&& fn) const {
    if (n) fn(0, n);
  }
};

// CSR offsets over `count` entries of random lengths in [lo, hi]; returns the blob bytes
uint64_t fill_off(Rng& r, Arr<uint64_t>& off, uint64_t count, uint64_t lo, uint64_t hi) {
  off.make(count + 1);
  uint64_t x = 0;
  for (uint64_t i = 0; i < count; i++) {
    off.p[i] = x;
    x += lo + r.below(hi - lo + 1);
  }
  off.p[count] = x;
  return x;
}

void fill_blob(Rng& r, Arr<uint8_t>& b, uint64_t bytes) {
  b.make(bytes);
  for (uint64_t i = 0; i < bytes; i++) b.p[i] = (uint8_t)r.next();
}

// one mutation of an offset array (entries [0, n]) bounded by `limit`
void mutate_off(Rng& r, Arr<uint64_t>& off, uint64_t limit) {
  if (off.n == 0) return;
  const uint64_t i = r.below(off.n);
  uint64_t& v = off.p[i];
  switch (r.below(7)) {
    case 0: v = 0; break;
    case 1: v += 1 + r.below(5); break;
    case 2: v = v > 5 ? v - 1 - r.below(5) : 0; break;
    case 3: v = limit + r.below(2); break;
    case 4: v = UINT64_MAX - r.below(3); break;
    case 5: v = r.next(); break;
    default:
      if (i + 1 < off.n) std::swap(off.p[i], off.p[i + 1]);
      break;
  }
}

// contract: off[a..b] non-decreasing and off[b] <= limit (ground truth, no shortcuts)
bool truth(const Arr<uint64_t>& off, uint64_t a, uint64_t b, uint64_t limit) {
  if (b < a || b >= off.n) return false;
  for (uint64_t i = a; i < b; i++)
    if (off.p[i] > off.p[i + 1]) return false;
  return off.p[b] <= limit;
}

volatile uint64_t g_sink = 0;
void touch(const uint8_t* p, uint64_t n) {  // read every byte of a range (ASan checks it)
  uint64_t s = 0;
  for (uint64_t i = 0; i < n; i++) s += p[i];
  g_sink = g_sink + s;
}

struct Stats {
  uint64_t sig_batches = 0, sig_invalid = 0, sig_lanes_packed = 0, tx_batches = 0, tx_invalid = 0, comp_batches = 0,
           comp_invalid = 0, ftx_batches = 0, ftx_invalid = 0;
};

struct MsgV {  // the generic batch's message view (runtime.hpp MsgView, host CSR)
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* tx_of = nullptr;
  const uint8_t* ptr(uint64_t i) const { return base + off[i]; }
  uint64_t len(uint64_t i) const { return off[i + 1] - off[i]; }
};

bool sig_round(Rng& r, Stats& st) {
  const uint64_t n = 1 + r.below(300);
  Arr<uint8_t> scheme, key, sig, msg, status;
  Arr<uint64_t> ko, so, mo;
  scheme.make(n);
  status.make(n);
  ko.make(n + 1), so.make(n + 1), mo.make(n + 1);
  uint64_t kx = 0, sx = 0, mx = 0;
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t c = r.below(10);
    const uint8_t sc = c < 5 ? CORDAHIP_SCHEME_EDDSA_ED25519_SHA512
                     : c < 7 ? CORDAHIP_SCHEME_ECDSA_SECP256R1_SHA256
                     : c < 9 ? CORDAHIP_SCHEME_ECDSA_SECP256K1_SHA256 : (uint8_t)r.below(8);
    scheme.p[i] = sc;
    const uint64_t kl = sc == CORDAHIP_SCHEME_EDDSA_ED25519_SHA512 ? (r.chance(90) ? 32 : r.below(70))
                        : (r.chance(90) ? (r.chance(50) ? 33 : 65) : r.below(70));
    const uint64_t sl = sc == CORDAHIP_SCHEME_EDDSA_ED25519_SHA512 ? (r.chance(90) ? 64 : r.below(80)) : r.below(90);
    const uint64_t ml = r.chance(80) ? 32 : r.below(100);
    ko.p[i] = kx, so.p[i] = sx, mo.p[i] = mx;
    kx += kl, sx += sl, mx += ml;
  }
  ko.p[n] = kx, so.p[n] = sx, mo.p[n] = mx;
  fill_blob(r, key, kx);
  fill_blob(r, sig, sx);
  fill_blob(r, msg, mx);
  uint64_t kb = kx, sb = sx, mb = mx;
  if (r.chance(75)) {
    for (int m = 0, nm = 1 + (int)r.below(3); m < nm; m++) {
      switch (r.below(5)) {
        case 0: mutate_off(r, ko, kx); break;
        case 1: mutate_off(r, so, sx); break;
        case 2: mutate_off(r, mo, mx); break;
        default: {  // a declared length short of the blob's use
          uint64_t& d = r.chance(34) ? kb : r.chance(50) ? sb : mb;
          d = d ? d - 1 - r.below(d < 8 ? d : 8) : 0;
        }
      }
    }
  }
  const bool valid = truth(ko, 0, n, kb) && truth(so, 0, n, sb) && truth(mo, 0, n, mb);
  const cordahip_sig_batch b{n, scheme.get(), key.get(), ko.get(), sig.get(), so.get(), msg.get(), mo.get(),
                             status.get(), nullptr, 0u, kb, sb, mb};
  const MsgV mv{msg.get(), mo.get()};
  // the pipeline's order of work: chunk by chunk, classify every lane, pack only a clean chunk
  bool failed = false;
  std::vector<uint16_t> cls;
  std::vector<uint64_t> mlen;
  std::vector<uint8_t> rk(32), rs(64), rm, rp(1), hsc(1), hk(65), hkl(1), hs(72), hsl(1), hm, hpre(1);
  uint64_t hmo[1];
  for (uint64_t a = 0; a < n && !failed;) {
    const uint64_t m = std::min<uint64_t>(n - a, 1 + r.below(64));
    cls.assign(m, 0);
    mlen.assign(m, 0);
    for (uint64_t q = 0; q < m; q++) {
      cls[q] = classify(&b, mv, a + q, mlen[q]);
      if (cls[q] == kBadCsr) failed = true;
    }
    if (failed) break;
    for (uint64_t q = 0; q < m; q++) {
      const uint64_t i = a + q;
      if (cls[q] == kEdBase) {
        rm.assign(mlen[q] ? mlen[q] : 1, 0);
        pack_ed_row(&b, mv, true, i, (uint32_t)mlen[q], rk.data(), rs.data(), mlen[q] ? rm.data() : nullptr, rp.data());
        st.sig_lanes_packed++;
      } else if (cls[q] == kEc) {
        hm.assign(mlen[q] ? mlen[q] : 1, 0);
        uint64_t mo0 = 0;
        pack_ec_row(&b, mv, true, i, 0, hsc.data(), hk.data(), hkl.data(), hs.data(), hsl.data(), hm.data(), hmo,
                    hpre.data(), mo0, nullptr);
        st.sig_lanes_packed++;
      }
    }
    a += m;
  }
  st.sig_batches++;
  st.sig_invalid += failed;
  if (failed == valid) {
    fprintf(stderr, "generic batch: classify says %s, the contract %s (n %llu)\n", failed ? "invalid" : "valid",
            valid ? "valid" : "invalid", (unsigned long long)n);
    return false;
  }
  return true;
}

bool tx_round(Rng& r, Stats& st) {
  const uint64_t ntx = r.below(60);
  Arr<uint64_t> tlo, lo, tso, ko, so;
  Arr<uint8_t> leaves, key, sig;
  uint64_t nleaves = fill_off(r, tlo, ntx, 0, 6);
  const uint64_t lb = fill_off(r, lo, nleaves, 0, 40);
  fill_blob(r, leaves, lb);
  uint64_t nsig = fill_off(r, tso, ntx, 0, 3);
  const uint64_t kx = fill_off(r, ko, nsig, 32, 32), sx = fill_off(r, so, nsig, 64, 64);
  fill_blob(r, key, kx);
  fill_blob(r, sig, sx);
  uint64_t lbl = lb, kb = kx, sb = sx, nl = nleaves, ns = nsig;
  if (r.chance(75)) {
    switch (r.below(9)) {
      case 0: mutate_off(r, tlo, nleaves); break;
      case 1: mutate_off(r, lo, lb); break;
      case 2: mutate_off(r, tso, nsig); break;
      case 3: mutate_off(r, ko, kx); break;
      case 4: mutate_off(r, so, sx); break;
      case 5: nl = nl ? nl - 1 : 0; break;
      case 6: ns = ns ? ns - 1 : 0; break;
      case 7: lbl = lbl ? lbl - 1 - r.below(lbl < 4 ? lbl : 4) : 0; break;
      default: kb = kb ? kb - 1 : 0; break;
    }
  }
  // the contract (nl / ns are the declared counts: the arrays hold nl + 1 / ns + 1 entries of
  // which the library may read only those)
  bool valid = true;
  if (ntx) {
    valid = nl + 1 <= lo.n && ns + 1 <= ko.n && truth(tlo, 0, ntx, nl) && truth(lo, tlo.p[0], tlo.p[ntx], lbl) &&
            truth(tso, 0, ntx, ns) &&
            (tso.p[0] == tso.p[ntx] || (truth(ko, tso.p[0], tso.p[ntx], kb) && truth(so, tso.p[0], tso.p[ntx], sb)));
  }
  // the library's view: arrays cut to their declared counts (a read past them is a report)
  Arr<uint64_t> lo_d, ko_d, so_d;
  auto cut = [](const Arr<uint64_t>& src, Arr<uint64_t>& dst, uint64_t count) {
    dst.make(std::min<uint64_t>(src.n, count + 1));
    if (dst.n) std::memcpy(dst.p.get(), src.p.get(), dst.n * 8);
  };
  cut(lo, lo_d, nl);
  cut(ko, ko_d, ns);
  cut(so, so_d, ns);
  Arr<uint8_t> txid, txst;
  txid.make(ntx * 32);
  txst.make(ntx);
  cordahip_txid_batch tb{ntx, leaves.get(), lo_d.get(), tlo.get(), txid.get(), txst.get(), nl, lbl};
  const SerialPar par;
  const bool ok = check_txid_batch(par, &tb) &&
                  check_sig_level(par, ntx, tso.get(), ns, ko_d.get(), kb, so_d.get(), sb);
  st.tx_batches++;
  st.tx_invalid += !ok;
  if (ok != valid) {
    fprintf(stderr, "tx batch: checks say %s, the contract %s (ntx %llu)\n", ok ? "valid" : "invalid",
            valid ? "valid" : "invalid", (unsigned long long)ntx);
    return false;
  }
  if (ok && ntx) {  // walk it as the library does: every leaf and every signature's key and sig
    for (uint64_t t = 0; t < ntx; t++) {
      for (uint64_t l = tlo.p[t]; l < tlo.p[t + 1]; l++) touch(leaves.p.get() + lo_d.p[l], lo_d.p[l + 1] - lo_d.p[l]);
      for (uint64_t q = tso.p[t]; q < tso.p[t + 1]; q++) {
        touch(key.p.get() + ko_d.p[q], ko_d.p[q + 1] - ko_d.p[q]);
        touch(sig.p.get() + so_d.p[q], so_d.p[q + 1] - so_d.p[q]);
      }
    }
  }
  return true;
}

bool comp_round(Rng& r, Stats& st) {
  const uint64_t ntx = r.below(60);
  Arr<uint64_t> tio;
  uint64_t nitems = fill_off(r, tio, ntx, 0, 7), ni = nitems;
  Arr<cordahip_kryo_item> items;
  if (r.chance(75)) {
    if (r.chance(70)) mutate_off(r, tio, nitems);
    else ni = ni ? ni - 1 - r.below(ni < 3 ? ni : 3) : 0;
  }
  items.make(ni);  // the library's view: exactly the declared records
  const bool valid = ntx == 0 || truth(tio, 0, ntx, ni);
  cordahip_txcomp_batch c{ntx, items.get(), tio.get(), nullptr, 0, nullptr, nullptr, ni};
  const bool ok = check_txcomp_batch(SerialPar{}, &c);
  st.comp_batches++;
  st.comp_invalid += !ok;
  if (ok != valid) {
    fprintf(stderr, "component batch: check says %s, the contract %s\n", ok ? "valid" : "invalid",
            valid ? "valid" : "invalid");
    return false;
  }
  if (ok && ntx)
    for (uint64_t t = 0; t < ntx; t++)
      for (uint64_t i = tio.p[t]; i < tio.p[t + 1]; i++) g_sink = g_sink + items.p[i].len;
  return true;
}

bool ftx_round(Rng& r, Stats& st) {
  const uint64_t ntx = r.below(40);
  Arr<uint64_t> tlo, lo, tko;
  Arr<uint8_t> leaves, tok, tok_hash, root, txst;
  uint64_t nleaves = fill_off(r, tlo, ntx, 0, 5);
  const uint64_t lb = fill_off(r, lo, nleaves, 0, 30);
  fill_blob(r, leaves, lb);
  uint64_t ntok = fill_off(r, tko, ntx, 1, 9);
  uint64_t nl = nleaves, nt = ntok, lbl = lb;
  if (r.chance(75)) {
    switch (r.below(6)) {
      case 0: mutate_off(r, tlo, nleaves); break;
      case 1: mutate_off(r, lo, lb); break;
      case 2: mutate_off(r, tko, ntok); break;
      case 3: nl = nl ? nl - 1 : 0; break;
      case 4: nt = nt ? nt - 1 : 0; break;
      default: lbl = lbl ? lbl - 1 : 0; break;
    }
  }
  bool valid = true;
  if (ntx)
    valid = truth(tlo, 0, ntx, nl) && truth(lo, tlo.p[0], tlo.p[ntx], lbl) && truth(tko, 0, ntx, nt);
  Arr<uint64_t> lo_d;
  lo_d.make(std::min<uint64_t>(lo.n, nl + 1));
  if (lo_d.n) std::memcpy(lo_d.p.get(), lo.p.get(), lo_d.n * 8);
  tok.make(nt);
  tok_hash.make(nt * 32);
  root.make(ntx * 32);
  txst.make(ntx);
  cordahip_filtered_tx_batch b{ntx, leaves.get(), lo_d.get(), tlo.get(), tok.get(), tok_hash.get(), tko.get(),
                               root.get(), txst.get(), nl, lbl, nt};
  const bool ok = check_filtered_batch(SerialPar{}, &b);
  st.ftx_batches++;
  st.ftx_invalid += !ok;
  if (ok != valid) {
    fprintf(stderr, "filtered batch: check says %s, the contract %s\n", ok ? "valid" : "invalid",
            valid ? "valid" : "invalid");
    return false;
  }
  if (ok && ntx)
    for (uint64_t t = 0; t < ntx; t++) {
      for (uint64_t l = tlo.p[t]; l < tlo.p[t + 1]; l++) touch(leaves.p.get() + lo_d.p[l], lo_d.p[l + 1] - lo_d.p[l]);
      touch(tok.p.get() + tko.p[t], tko.p[t + 1] - tko.p[t]);
      touch(tok_hash.p.get() + 32 * tko.p[t], 32 * (tko.p[t + 1] - tko.p[t]));
    }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: csr_fuzz ROUNDS RNG_SEED\n");
    return 2;
  }
  const uint64_t rounds = strtoull(argv[1], nullptr, 10);
  Rng r{strtoull(argv[2], nullptr, 10)};
  Stats st;
  for (uint64_t k = 0; k < rounds; k++)
    if (!sig_round(r, st) || !tx_round(r, st) || !comp_round(r, st) || !ftx_round(r, st)) return 1;
  printf("{\"rounds\": %llu, \"sig_batches\": %llu, \"sig_invalid\": %llu, \"sig_lanes_packed\": %llu, "
         "\"tx_batches\": %llu, \"tx_invalid\": %llu, \"comp_batches\": %llu, \"comp_invalid\": %llu, "
         "\"ftx_batches\": %llu, \"ftx_invalid\": %llu}\n",
         (unsigned long long)rounds, (unsigned long long)st.sig_batches, (unsigned long long)st.sig_invalid,
         (unsigned long long)st.sig_lanes_packed, (unsigned long long)st.tx_batches, (unsigned long long)st.tx_invalid,
         (unsigned long long)st.comp_batches, (unsigned long long)st.comp_invalid, (unsigned long long)st.ftx_batches,
         (unsigned long long)st.ftx_invalid);
  return 0;
}

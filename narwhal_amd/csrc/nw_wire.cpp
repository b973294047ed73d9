// nw_wire.cpp — wire-format ingest: bincode-serialized
// primary::PrimaryMessage frames, as the primary's network receiver gets them
// (PrimaryReceiverHandler::dispatch, primary/src/primary.rs:224-240:
// `bincode::deserialize(&serialized)`), decoded natively into the structure-of-arrays the
// verification pipelines take, then verified with the check the primary applies to each
// variant (Header::verify, Vote::verify, Certificate::verify; primary/src/messages.rs).
//
// Wire format (bincode 1.3 `serialize`/`deserialize`: fixint little-endian, u64 lengths,
// trailing bytes allowed; serde derives in primary/src/messages.rs and crypto/src/lib.rs):
//   PrimaryMessage  u32 variant: 0 Header, 1 Vote, 2 Certificate, 3 CertificatesRequest
//   Header          author PK | round u64 | payload: u64 n, n x (Digest 32 | WorkerId u32)
//                   | parents: u64 n, n x Digest 32 | id Digest 32 | signature 64
//   Vote            id 32 | round u64 | origin PK | author PK | signature 64
//   Certificate     Header | votes: u64 n, n x (PK | signature 64)
//   PK (PublicKey)  serde string: u64 len | base64 text (crypto/src/lib.rs:94-112), decoded
//                   with base64 0.13 STANDARD (padding optional, non-zero trailing bits
//                   rejected) and then sliced [..32] (lib.rs:73-79: longer decodings keep
//                   their first 32 bytes; shorter ones panic in the reference, here they are
//                   a serialization error)
//   Digest          32 raw bytes (newtype over [u8; 32]); Signature: part1 32 | part2 32
// Deserialising into BTreeMap / BTreeSet sorts the entries and drops duplicate keys (the
// last value wins in the map), so the `Hash for Header` bytes (messages.rs:70-84) are built
// from the sorted, de-duplicated payload and parents, exactly as the reference hashes the
// value it deserialised.
#include <string.h>

#include <algorithm>
#include <functional>
#include <thread>
#include <utility>
#include <vector>

#include "narwhal_amd.h"
#include "nw_runtime.h"

namespace {

using nw::rt::set_err;

struct Reader {
  const uint8_t* p;
  size_t n, pos = 0;
  bool ok = true;
  const uint8_t* take(size_t k) {
    if (!ok || k > n - pos) {
      ok = false;
      return nullptr;
    }
    const uint8_t* r = p + pos;
    pos += k;
    return r;
  }
  uint32_t u32() {
    const uint8_t* b = take(4);
    uint32_t v = 0;
    if (b) memcpy(&v, b, 4);
    return v;
  }
  uint64_t u64() {
    const uint8_t* b = take(8);
    uint64_t v = 0;
    if (b) memcpy(&v, b, 8);
    return v;
  }
  void raw(uint8_t* out, size_t k) {
    const uint8_t* b = take(k);
    if (b) memcpy(out, b, k);
  }
  // Sequence length that cannot exceed the remaining bytes at `elem` bytes per element.
  uint64_t len(size_t elem) {
    const uint64_t v = u64();
    if (ok && elem && v > (n - pos) / elem) ok = false;
    return ok ? v : 0;
  }
};

int b64_value(uint8_t c) {
  if (c >= 'A' && c <= 'Z') return c - 'A';
  if (c >= 'a' && c <= 'z') return c - 'a' + 26;
  if (c >= '0' && c <= '9') return c - '0' + 52;
  if (c == '+') return 62;
  if (c == '/') return 63;
  return -1;
}

// base64 0.13 STANDARD decode of s[0..len): validates the whole string, keeps the first
// 32 decoded bytes in out32 and returns the decoded length (-1 if invalid).
long b64_decode32(const uint8_t* s, size_t len, uint8_t out32[32]) {
  size_t end = len;
  int pad = 0;
  while (end > 0 && s[end - 1] == '=' && pad < 2) {
    --end;
    ++pad;
  }
  if (pad && (len % 4) != 0) return -1;             // padded input comes in whole quads
  if (end % 4 == 1) return -1;                      // a lone trailing symbol
  if (pad && (end % 4) + pad != 4) return -1;       // padding must complete the last quad
  uint32_t acc = 0;
  int bits = 0;
  long nout = 0;
  for (size_t i = 0; i < end; ++i) {
    const int v = b64_value(s[i]);
    if (v < 0) return -1;
    acc = (acc << 6) | (uint32_t)v;
    bits += 6;
    if (bits >= 8) {
      bits -= 8;
      if (nout < 32) out32[nout] = (uint8_t)(acc >> bits);
      ++nout;
      acc &= (1u << bits) - 1;
    }
  }
  return acc == 0 ? nout : -1;                      // non-zero trailing bits rejected
}

bool read_pk(Reader& r, uint8_t out[32]) {
  const uint64_t L = r.len(1);
  const uint8_t* s = r.take(L);
  if (!r.ok) return false;
  if (b64_decode32(s, L, out) < 32) return (r.ok = false);
  return true;
}

struct Digest32 {
  uint8_t b[32];
  bool operator<(const Digest32& o) const { return memcmp(b, o.b, 32) < 0; }
  bool operator==(const Digest32& o) const { return memcmp(b, o.b, 32) == 0; }
};

// One decoded header: appends its `Hash for Header` bytes, id and signature.
struct HeaderSoA {
  std::vector<uint8_t> bytes, ids, sigs;
  std::vector<uint64_t> offsets{0};
  std::vector<uint32_t> payload_counts;
  size_t n() const { return payload_counts.size(); }
  void clear() {   // sizes only: the capacity is kept for the next call
    bytes.clear();
    ids.clear();
    sigs.clear();
    offsets.assign(1, 0);
    payload_counts.clear();
  }
};

// Per-thread scratch, reused across frames (no allocation on the steady path).
struct Scratch {
  std::vector<std::pair<Digest32, uint32_t>> pay, upay;
  std::vector<Digest32> par;
};

// Appends one header to h only if it decodes completely.
bool read_header(Reader& r, HeaderSoA& h, Scratch& sc) {
  uint8_t author[32];
  if (!read_pk(r, author)) return false;
  const uint64_t round = r.u64();
  const uint64_t np = r.len(36);
  sc.pay.resize(np);
  for (uint64_t i = 0; i < np && r.ok; ++i) {
    r.raw(sc.pay[i].first.b, 32);
    sc.pay[i].second = r.u32();
  }
  const uint64_t nq = r.len(32);
  sc.par.resize(nq);
  for (uint64_t i = 0; i < nq && r.ok; ++i) r.raw(sc.par[i].b, 32);
  uint8_t id[32], sig[64];
  r.raw(id, 32);
  r.raw(sig, 64);
  if (!r.ok) return false;
  // BTreeMap: sorted, duplicate keys keep the last value; BTreeSet: sorted, unique.
  auto& pay = sc.pay;
  auto& upay = sc.upay;
  auto key_less = [](const auto& x, const auto& y) { return x.first < y.first; };
  if (!std::is_sorted(pay.begin(), pay.end(), key_less))   // wire order is usually sorted
    std::stable_sort(pay.begin(), pay.end(), key_less);
  upay.clear();
  for (size_t i = 0; i < pay.size(); ++i) {
    if (!upay.empty() && upay.back().first == pay[i].first) upay.back().second = pay[i].second;
    else upay.push_back(pay[i]);
  }
  auto& par = sc.par;
  if (!std::is_sorted(par.begin(), par.end())) std::sort(par.begin(), par.end());
  par.erase(std::unique(par.begin(), par.end()), par.end());
  auto& B = h.bytes;
  const size_t at = B.size();
  B.resize(at + 40 + 36 * upay.size() + 32 * par.size());
  uint8_t* o = B.data() + at;
  memcpy(o, author, 32);
  memcpy(o + 32, &round, 8);
  o += 40;
  for (const auto& e : upay) {
    memcpy(o, e.first.b, 32);
    memcpy(o + 32, &e.second, 4);
    o += 36;
  }
  for (const auto& d : par) {
    memcpy(o, d.b, 32);
    o += 32;
  }
  h.offsets.push_back(B.size());
  h.payload_counts.push_back((uint32_t)upay.size());
  h.ids.insert(h.ids.end(), id, id + 32);
  h.sigs.insert(h.sigs.end(), sig, sig + 64);
  return true;
}

void pop_header(HeaderSoA& h) {
  h.offsets.pop_back();
  h.bytes.resize(h.offsets.back());
  h.payload_counts.pop_back();
  h.ids.resize(h.ids.size() - 32);
  h.sigs.resize(h.sigs.size() - 64);
}

nw_certificates view(const HeaderSoA& h, const std::vector<uint64_t>* vote_offsets,
                     const std::vector<uint8_t>* vpk, const std::vector<uint8_t>* vsig) {
  nw_certificates c{};
  c.n = h.n();
  c.header_bytes = h.bytes.data();
  c.header_offsets = h.offsets.data();
  c.payload_counts = h.payload_counts.data();
  c.ids = h.ids.data();
  c.header_sigs = h.sigs.data();
  if (vote_offsets) {
    c.vote_offsets = vote_offsets->data();
    c.vote_pks = vpk->data();
    c.vote_sigs = vsig->data();
    c.nvotes = vote_offsets->back();
  }
  c.header_bytes_len = h.bytes.size();
  return c;
}

// All frames decoded into per-variant structure-of-arrays (+ the frame of each item).
struct Decoded {
  HeaderSoA hdr, cert;
  std::vector<uint64_t> hdr_of, cert_of, vote_of;
  std::vector<uint64_t> cvo{0};
  std::vector<uint8_t> cvpk, cvsig;
  std::vector<uint8_t> v_ids, v_origins, v_authors, v_sigs;
  std::vector<uint64_t> v_rounds;
  void clear() {
    hdr.clear();
    cert.clear();
    hdr_of.clear();
    cert_of.clear();
    vote_of.clear();
    cvo.assign(1, 0);
    cvpk.clear();
    cvsig.clear();
    v_ids.clear();
    v_origins.clear();
    v_authors.clear();
    v_sigs.clear();
    v_rounds.clear();
  }
};

// Decodes frame i into d; returns its NW_MSG_* kind or -1 (d unchanged then). counts
// (optional, 3 values): payload entries and parents after BTreeMap/BTreeSet
// de-duplication, votes.
int32_t decode_frame(const uint8_t* f, size_t len, uint64_t i, Decoded& d, uint64_t* counts,
                     Scratch& sc) {
  Reader r{f, len};
  const uint32_t variant = r.u32();
  if (!r.ok || variant > NW_MSG_CERTIFICATES_REQUEST) return -1;
  if (counts) counts[0] = counts[1] = counts[2] = 0;
  if (variant == NW_MSG_HEADER || variant == NW_MSG_CERTIFICATE) {
    HeaderSoA& h = variant == NW_MSG_HEADER ? d.hdr : d.cert;
    if (!read_header(r, h, sc)) return -1;
    const uint64_t hl = h.offsets.back() - h.offsets[h.offsets.size() - 2];
    const uint64_t np = h.payload_counts.back();
    if (counts) {
      counts[0] = np;
      counts[1] = (hl - 40 - 36 * np) / 32;
    }
    if (variant == NW_MSG_HEADER) {
      d.hdr_of.push_back(i);
      return NW_MSG_HEADER;
    }
    const uint64_t nv = r.len(72);   // each vote >= 8-byte length + 64-byte signature
    const size_t pk0 = d.cvpk.size(), sg0 = d.cvsig.size();
    if (r.ok) {
      d.cvpk.resize(pk0 + 32 * nv);
      d.cvsig.resize(sg0 + 64 * nv);
      for (uint64_t v = 0; v < nv && r.ok; ++v) {
        if (read_pk(r, &d.cvpk[pk0 + 32 * v])) r.raw(&d.cvsig[sg0 + 64 * v], 64);
      }
    }
    if (!r.ok) {
      pop_header(d.cert);
      d.cvpk.resize(pk0);
      d.cvsig.resize(sg0);
      return -1;
    }
    if (counts) counts[2] = nv;
    d.cvo.push_back(d.cvo.back() + nv);
    d.cert_of.push_back(i);
    return NW_MSG_CERTIFICATE;
  }
  if (variant == NW_MSG_VOTE) {
    uint8_t id[32], origin[32], author[32], sig[64];
    r.raw(id, 32);
    const uint64_t round = r.u64();
    if (!r.ok || !read_pk(r, origin) || !read_pk(r, author)) return -1;
    r.raw(sig, 64);
    if (!r.ok) return -1;
    d.v_ids.insert(d.v_ids.end(), id, id + 32);
    d.v_rounds.push_back(round);
    d.v_origins.insert(d.v_origins.end(), origin, origin + 32);
    d.v_authors.insert(d.v_authors.end(), author, author + 32);
    d.v_sigs.insert(d.v_sigs.end(), sig, sig + 64);
    d.vote_of.push_back(i);
    return NW_MSG_VOTE;
  }
  // CertificatesRequest(Vec<Digest>, PublicKey): decoded for well-formedness only.
  const uint64_t nd = r.len(32);
  r.take(32 * nd);
  uint8_t pk[32];
  if (!r.ok || !read_pk(r, pk)) return -1;
  if (counts) counts[0] = nd;
  return NW_MSG_CERTIFICATES_REQUEST;
}

// Decodes all frames, in parallel over contiguous ranges (host threads; the per-range
// results are merged in frame order, in place and in parallel).
void decode_all(const uint8_t* frames, const uint64_t* offsets, size_t n, Decoded& d,
                int32_t* kind_out, uint64_t* counts_out) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t T = std::min<size_t>({(size_t)std::min(hw, 16u), (n + 4095) / 4096, 64});
  auto run = [&](size_t a, size_t b, Decoded& out) {
    Scratch sc;
    for (size_t i = a; i < b; ++i)
      kind_out[i] = decode_frame(frames + offsets[i], (size_t)(offsets[i + 1] - offsets[i]), i,
                                 out, counts_out ? counts_out + 3 * i : nullptr, sc);
  };
  if (T <= 1) {
    run(0, n, d);
    return;
  }
  // The per-range outputs persist per calling thread: their capacity is reused by the next
  // call, so the decode does not page-fault freshly grown vectors in every call (65,536
  // frames: 47 ms -> ~9 ms on 8 threads; the faults serialize on the address space).
  thread_local std::vector<Decoded> parts;
  if (parts.size() < T) parts.resize(T);
  std::vector<std::thread> th;
  for (size_t t = 0; t < T; ++t) {
    parts[t].clear();
    th.emplace_back(run, n * t / T, n * (t + 1) / T, std::ref(parts[t]));
  }
  for (auto& x : th) x.join();
  // merge in parallel: size the merged arrays once, then every part copies its slices into
  // place (offset arrays rebased by the bytes / votes of the earlier parts)
  struct Job {
    void* dst;
    const void* src;
    size_t bytes;
    uint64_t add;   // != 0: uint64 elements, each + add
  };
  std::vector<std::vector<Job>> jobs(T);
  auto plan = [&](auto get) {   // get(Decoded&) -> std::vector<X>& (plain concatenation)
    size_t tot = 0;
    for (size_t t = 0; t < T; ++t) tot += get(parts[t]).size();
    auto& dv = get(d);
    const size_t at = dv.size();
    dv.resize(at + tot);
    size_t o = at;
    for (size_t t = 0; t < T; ++t) {
      auto& sv = get(parts[t]);
      using X = typename std::decay_t<decltype(sv)>::value_type;
      if (!sv.empty()) jobs[t].push_back({dv.data() + o, sv.data(), sv.size() * sizeof(X), 0});
      o += sv.size();
    }
  };
  auto plan_offsets = [&](auto get, auto base_of) {   // [0, a, b, ...] arrays: skip the 0
    size_t tot = 0;
    for (size_t t = 0; t < T; ++t) tot += get(parts[t]).size() - 1;
    auto& dv = get(d);
    size_t o = dv.size();
    uint64_t base = dv.back();
    dv.resize(o + tot);
    for (size_t t = 0; t < T; ++t) {
      auto& sv = get(parts[t]);
      if (sv.size() > 1)
        jobs[t].push_back({dv.data() + o, sv.data() + 1, (sv.size() - 1) * 8, base + 1});
      o += sv.size() - 1;
      base += base_of(parts[t]);
    }
  };
  for (int hc = 0; hc < 2; ++hc) {
    auto H = [hc](Decoded& x) -> HeaderSoA& { return hc ? x.cert : x.hdr; };
    plan_offsets([&](Decoded& x) -> std::vector<uint64_t>& { return H(x).offsets; },
                 [&](Decoded& x) { return (uint64_t)H(x).bytes.size(); });
    plan([&](Decoded& x) -> std::vector<uint8_t>& { return H(x).bytes; });
    plan([&](Decoded& x) -> std::vector<uint32_t>& { return H(x).payload_counts; });
    plan([&](Decoded& x) -> std::vector<uint8_t>& { return H(x).ids; });
    plan([&](Decoded& x) -> std::vector<uint8_t>& { return H(x).sigs; });
  }
  plan_offsets([](Decoded& x) -> std::vector<uint64_t>& { return x.cvo; },
               [](Decoded& x) { return x.cvo.back(); });
  plan([](Decoded& x) -> std::vector<uint64_t>& { return x.hdr_of; });
  plan([](Decoded& x) -> std::vector<uint64_t>& { return x.cert_of; });
  plan([](Decoded& x) -> std::vector<uint64_t>& { return x.vote_of; });
  plan([](Decoded& x) -> std::vector<uint8_t>& { return x.cvpk; });
  plan([](Decoded& x) -> std::vector<uint8_t>& { return x.cvsig; });
  plan([](Decoded& x) -> std::vector<uint8_t>& { return x.v_ids; });
  plan([](Decoded& x) -> std::vector<uint8_t>& { return x.v_origins; });
  plan([](Decoded& x) -> std::vector<uint8_t>& { return x.v_authors; });
  plan([](Decoded& x) -> std::vector<uint8_t>& { return x.v_sigs; });
  plan([](Decoded& x) -> std::vector<uint64_t>& { return x.v_rounds; });
  th.clear();
  for (size_t t = 0; t < T; ++t)
    th.emplace_back([&jobs, t] {
      for (const Job& j : jobs[t]) {
        if (!j.add) {
          memcpy(j.dst, j.src, j.bytes);
          continue;
        }
        uint64_t* o = static_cast<uint64_t*>(j.dst);
        const uint64_t* i = static_cast<const uint64_t*>(j.src);
        for (size_t k = 0; k < j.bytes / 8; ++k) o[k] = i[k] + (j.add - 1);
      }
    });
  for (auto& x : th) x.join();
}

int check_frames(const uint8_t* frames, const uint64_t* offsets, size_t n) {
  if (n && (!frames || !offsets)) return set_err(NW_E_INVALID_ARG, "null pointer");
  for (size_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return set_err(NW_E_INVALID_ARG, "offsets not monotone");
  return 0;
}

}  // namespace

extern "C" {

int nw_primary_messages_scan(const uint8_t* frames, const uint64_t* offsets, size_t n,
                             int32_t* kind_out, uint64_t* counts_out) {
  int rc = check_frames(frames, offsets, n);
  if (rc) return rc;
  if (n && !kind_out) return set_err(NW_E_INVALID_ARG, "null kind_out");
  thread_local Decoded d;
  d.clear();
  decode_all(frames, offsets, n, d, kind_out, counts_out);
  return 0;
}

int nw_primary_messages_verify_wire(const nw_committee* committee, const uint8_t* frames,
                                    const uint64_t* offsets, size_t n, int32_t* kind_out,
                                    int32_t* status_out, uint64_t* index_out) {
  int rc = nw::rt::ensure_init();
  if (rc) return rc;
  rc = check_frames(frames, offsets, n);
  if (rc) return rc;
  if (n && !status_out) return set_err(NW_E_INVALID_ARG, "null status_out");
  thread_local Decoded d;
  d.clear();
  std::vector<int32_t> kinds(n);
  decode_all(frames, offsets, n, d, kinds.data(), nullptr);
  for (size_t i = 0; i < n; ++i) {
    status_out[i] = kinds[i] < 0 ? NW_DAG_SERIALIZATION : 0;
    if (index_out) index_out[i] = 0;
    if (kind_out) kind_out[i] = kinds[i];
  }
  std::vector<int32_t> st;
  std::vector<uint64_t> ix;
  auto scatter = [&](const std::vector<uint64_t>& of) {
    for (size_t k = 0; k < of.size(); ++k) {
      status_out[of[k]] = st[k];
      if (index_out) index_out[of[k]] = ix[k];
    }
  };
  if (d.hdr.n()) {
    st.assign(d.hdr.n(), 0);
    ix.assign(d.hdr.n(), 0);
    nw_certificates h = view(d.hdr, nullptr, nullptr, nullptr);
    rc = nw_headers_verify_many(committee, &h, st.data(), ix.data());
    if (rc < 0) return rc;
    scatter(d.hdr_of);
  }
  if (d.cert.n()) {
    st.assign(d.cert.n(), 0);
    ix.assign(d.cert.n(), 0);
    nw_certificates c = view(d.cert, &d.cvo, &d.cvpk, &d.cvsig);
    rc = nw_certificates_verify_many(committee, &c, nullptr, st.data(), ix.data());
    if (rc < 0) return rc;
    scatter(d.cert_of);
  }
  if (!d.vote_of.empty()) {
    st.assign(d.vote_of.size(), 0);
    ix.assign(d.vote_of.size(), 0);
    rc = nw_votes_verify_many(committee, d.v_ids.data(), d.v_rounds.data(), d.v_origins.data(),
                              d.v_authors.data(), d.v_sigs.data(), d.vote_of.size(), st.data());
    if (rc < 0) return rc;
    scatter(d.vote_of);
  }
  return 0;
}

}  // extern "C"

// Host-only check (no GPU) of the copy-on-write against live results (Index + ViewTracker): an
// index with a live view and one without take the same updates; every particle's lists must hold
// the same records in both, each index must pass Index::check, and what the view saw (the lists
// at publication) must be unchanged in the pool it points into.
//   make -C mqtt-server_amd build/cow_check && mqtt-server_amd/build/cow_check 40000
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <tuple>
#include <vector>

#include "index.h"

extern "C" {
void* mqgen_subs(uint64_t n_subs, uint32_t n_clients, uint64_t seed, int mix);
uint64_t mqgen_subs_n(void* h);
uint64_t mqgen_subs_nbytes(void* h);
void mqgen_subs_copy(void* h, uint8_t* bytes, uint64_t* offs, uint32_t* client_ids, uint32_t* filter_ids,
                     uint8_t* qos, uint8_t* flags, int32_t* idents);
void mqgen_subs_free(void* h);
}

using namespace mq;

// the records of every live particle's list, as a sorted multiset per node
static std::vector<std::vector<std::tuple<uint32_t, uint32_t, int32_t, uint32_t>>> lists_of(const Index& ix) {
  std::vector<std::vector<std::tuple<uint32_t, uint32_t, int32_t, uint32_t>>> out(ix.lists.size());
  for (size_t n = 0; n < ix.lists.size(); n++) {
    const NodeLists& L = ix.lists.h[n];
    for (uint32_t i = 0; i < L.n_direct + L.n_merge; i++) {
      const SubRec& r = ix.subs.m.h[L.sub_off + i];
      out[n].emplace_back(r.client, r.filter_id, r.ident, r.meta);
    }
    std::sort(out[n].begin(), out[n].end());
  }
  return out;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 40000;
  void* g = mqgen_subs(n, (uint32_t)std::max<uint64_t>(1, n / 13), 73, 0);
  const uint64_t m = mqgen_subs_n(g);
  std::vector<uint8_t> bytes(mqgen_subs_nbytes(g) + 16);
  std::vector<uint64_t> offs(m + 1);
  std::vector<uint32_t> cid(m), fid(m);
  std::vector<uint8_t> qos(m), flags(m), out_new(m);
  std::vector<int32_t> ident(m);
  mqgen_subs_copy(g, bytes.data(), offs.data(), cid.data(), fid.data(), qos.data(), flags.data(), ident.data());
  mqgen_subs_free(g);
  ViewTracker views;
  Index a(m, 0), b(m, 0);
  a.set_views(&views);
  a.subscribe_bulk(bytes.data(), offs.data(), cid.data(), fid.data(), qos.data(), flags.data(), ident.data(), m,
                   out_new.data());
  b.subscribe_bulk(bytes.data(), offs.data(), cid.data(), fid.data(), qos.data(), flags.data(), ident.data(), m,
                   out_new.data());
  int bad = 0;
  std::string why;
  for (int round = 0; round < 3; round++) {
    // a view at publication: its lists' records, read through the pool pointer it holds
    const uint64_t gen = views.publish();
    const SubRec* pool = a.subs.m.h.data();
    std::vector<NodeLists> seen(a.lists.h.begin(), a.lists.h.end());
    std::vector<std::vector<SubRec>> seen_recs(seen.size());
    for (size_t k = 0; k < seen.size(); k++)
      seen_recs[k].assign(pool + seen[k].sub_off, pool + seen[k].sub_off + seen[k].n_direct + seen[k].n_merge);
    // updates: a new client on '#', overwrites, removals, may-merge flips
    auto both = [&](auto&& f) {
      const int ra = f(a), rb = f(b);
      if (ra != rb) {
        std::printf("answers differ: %d %d\n", ra, rb);
        bad++;
      }
    };
    both([&](Index& x) { return x.subscribe("#", 999990 + round, 777, 2, 0, 0); });
    for (uint32_t i = 0; i < 400; i++) {
      const uint32_t k = (uint32_t)((i * 7919u + round * 104729u) % m);
      const std::string f((const char*)bytes.data() + offs[k], offs[k + 1] - offs[k]);
      if (i % 3 == 0) both([&](Index& x) { return x.unsubscribe(f, cid[k]); });
      else if (i % 3 == 1) both([&](Index& x) { return x.subscribe(f, cid[k], fid[k], (qos[k] + 1) % 3, flags[k], ident[k]); });
      else both([&](Index& x) { return x.subscribe("#", cid[k], 555, 1, 0, 0); });
    }
    if (!a.check(&why)) {
      std::printf("round %d: index with a view fails check: %s\n", round, why.c_str());
      bad++;
    }
    if (!b.check(&why)) {
      std::printf("round %d: index without views fails check: %s\n", round, why.c_str());
      bad++;
    }
    if (lists_of(a) != lists_of(b)) {
      std::printf("round %d: lists differ between the indexes\n", round);
      bad++;
    }
    for (size_t k = 0; k < seen.size(); k++)
      for (size_t i = 0; i < seen_recs[k].size(); i++) {
        const SubRec& x = pool[seen[k].sub_off + i];
        const SubRec& y = seen_recs[k][i];
        if (x.client != y.client || x.filter_id != y.filter_id || x.ident != y.ident || x.meta != y.meta) {
          if (bad < 20) std::printf("round %d: node %zu record %zu changed under the view\n", round, k, i);
          bad++;
        }
      }
    views.release(gen);
  }
  std::printf("%s (%d problems)\n", bad ? "FAILED" : "ok", bad);
  return bad ? 1 : 0;
}

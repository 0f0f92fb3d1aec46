// Host-only diagnosis (no GPU): partner links per pair-list slot — how many may-merge records a
// set pass could resolve from the list's own partner alone (one link) — over all pair lists and
// over the lists of the busiest particles (the hot wildcard lists every topic gathers).
//   make -C mqtt-server_amd build/merge_stats && mqtt-server_amd/build/merge_stats 10000000
#include <cstdio>
#include <cstdlib>
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

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1000000;
  void* g = mqgen_subs(n, (uint32_t)std::max<uint64_t>(1, n / 10), 0x6D716D61ull, 0);
  const uint64_t m = mqgen_subs_n(g);
  std::vector<uint8_t> bytes(mqgen_subs_nbytes(g) + 16);
  std::vector<uint64_t> offs(m + 1);
  std::vector<uint32_t> cid(m), fid(m);
  std::vector<uint8_t> qos(m), flags(m), out_new(m);
  std::vector<int32_t> ident(m);
  mqgen_subs_copy(g, bytes.data(), offs.data(), cid.data(), fid.data(), qos.data(), flags.data(), ident.data());
  mqgen_subs_free(g);
  Index ix(m, 0);
  ix.subscribe_bulk(bytes.data(), offs.data(), cid.data(), fid.data(), qos.data(), flags.data(), ident.data(), m,
                    out_new.data());
  ix.flush_merge();
  uint64_t hist[2][18] = {{0}};
  uint64_t slots[2] = {0, 0};
  for (size_t nd = 0; nd < ix.npair.size(); nd++) {
    const NodePair& P = ix.npair.h[nd];
    if (P.ent_mask == kNone) continue;
    const NodeLists& L = ix.lists.h[nd];
    const int hot = L.n_direct + L.n_merge >= 1000 ? 1 : 0;
    for (uint32_t i = 0; i <= P.ent_mask; i++) {
      const PairEnt& e = ix.pent.m.h[P.ent_off + i];
      if (e.h == kNone) continue;
      for (uint32_t j = 0; j < e.cnt; j++) {
        const uint32_t c = ix.plist.m.h[e.off + j].mp_cnt;
        hist[hot][c > 16 ? 17 : c]++;
        slots[hot]++;
      }
    }
  }
  for (int h = 0; h < 2; h++) {
    printf("%s lists: %llu slots; partner links per slot:", h ? "hot (>= 1000 subscriptions)" : "other",
           (unsigned long long)slots[h]);
    for (int c = 1; c < 18; c++)
      if (hist[h][c]) printf(" %s%d: %.1f%%", c == 17 ? ">" : "", c == 17 ? 16 : c, 100.0 * hist[h][c] / slots[h]);
    printf("\n");
  }
  return 0;
}

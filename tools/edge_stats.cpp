// Host-only diagnosis (no GPU): edges per level of their parent — how many edge slots the
// root's and level 1's children take (the walk's level-0 / level-1 probes), for staging them in LDS.
//   make -C mqtt-server_amd build/edge_stats && mqtt-server_amd/build/edge_stats 10000000
#include <cstdio>
#include <algorithm>
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
  std::vector<int> depth(ix.walk.size(), -1);
  depth[kRoot] = 0;
  // parents first: nodes are numbered in BFS order by the bulk build
  uint64_t per[8] = {0}, total = 0;
  for (size_t n = 0; n < ix.walk.size(); n++) {
    if (n == kRoot) continue;
    const uint32_t p = ix.walk.h[n].parent_flags & kParentMask;
    if (p >= depth.size() || depth[p] < 0) continue;
    depth[n] = depth[p] + 1;
  }
  for (size_t i = 0; i < ix.edges.size(); i++) {
    const EdgeSlot& e = ix.edges.h[i];
    if (e.parent == kEdgeEmpty || e.parent == kEdgeTomb) continue;
    total++;
    const int d = e.parent < depth.size() ? depth[e.parent] : -1;
    if (d >= 0 && d < 8) per[d]++;
  }
  printf("nodes %zu, edges %llu (table %zu slots, %.1f MB)\n", ix.walk.size(), (unsigned long long)total,
         ix.edges.size(), ix.edges.size() * sizeof(EdgeSlot) / 1e6);
  for (int d = 0; d < 8; d++) printf("  children of level-%d particles: %llu\n", d, (unsigned long long)per[d]);
  // probe distances of the stored edges from their home slots (the walk's hit probes), and the
  // run length from a key's home slot to the first empty slot (its miss probes)
  const uint64_t mask = ix.edges.size() - 1;
  uint64_t dsum = 0, dmax = 0, hist[5] = {0};
  for (size_t i = 0; i < ix.edges.size(); i++) {
    const EdgeSlot& e = ix.edges.h[i];
    if (e.parent == kEdgeEmpty || e.parent == kEdgeTomb) continue;
    const uint64_t d = (i - (edge_hash(e.parent, SegKey{e.k0, e.k1}) & mask)) & mask;
    dsum += d;
    dmax = std::max(dmax, d);
    hist[std::min<uint64_t>(d, 4)]++;
  }
  printf("probe distance: mean %.4f, max %llu; 0: %llu, 1: %llu, 2: %llu, 3: %llu, 4+: %llu\n",
         total ? (double)dsum / total : 0.0, (unsigned long long)dmax, (unsigned long long)hist[0],
         (unsigned long long)hist[1], (unsigned long long)hist[2], (unsigned long long)hist[3],
         (unsigned long long)hist[4]);
  return 0;
}

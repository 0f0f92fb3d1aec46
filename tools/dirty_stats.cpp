// Update-path diagnosis (host only, no GPU): which device-image arrays a churn of K unsubscribes
// + K subscribes dirties, in pages of Mirror::kPageBytes, i.e. what Device::sync would upload.
// Same churn as tools/bench_update.py: K random live subscriptions unsubscribed, then the same
// filters subscribed by K new clients.
//   make -C mqtt-server_amd build/dirty_stats && mqtt-server_amd/build/dirty_stats 1000000 1000
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
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

template <class T>
static size_t dirty_pages(const Mirror<T>& m) {
  size_t c = 0;
  for (uint64_t w : m.dirty) c += (size_t)__builtin_popcountll(w);
  return c;
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1000000;
  const uint64_t k = argc > 2 ? strtoull(argv[2], nullptr, 10) : 1000;
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
#define MIRRORS(X)                                                                                        \
  X(edges) X(walk) X(lists) X(msg) X(seginfo) X(segbytes) X(subs.m) X(mref) X(mpart.m) X(npair) X(pent.m) \
      X(plist.m) X(shr.m) X(inl.m) X(children.m)
#define CLEAR(a) ix.a.clear_dirty();
  MIRRORS(CLEAR)
  std::mt19937_64 r(7);
  uint32_t next_client = 0;
  for (uint32_t c : cid) next_client = std::max(next_client, c + 1);
  std::vector<uint64_t> pick(k);
  for (auto& p : pick) p = r() % m;
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t p : pick)
    ix.unsubscribe(std::string_view((const char*)bytes.data() + offs[p], offs[p + 1] - offs[p]), cid[p]);
  const auto t1 = std::chrono::steady_clock::now();
  for (uint64_t p : pick)
    ix.subscribe(std::string_view((const char*)bytes.data() + offs[p], offs[p + 1] - offs[p]), next_client++, fid[p],
                 qos[p], flags[p], ident[p]);
  const auto t2 = std::chrono::steady_clock::now();
  ix.flush_merge();
  const auto t3 = std::chrono::steady_clock::now();
  auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
  printf("{\"subs\": %llu, \"ops\": %llu, \"unsubscribe_ms\": %.2f, \"subscribe_ms\": %.2f, \"flush_merge_ms\": %.2f, "
         "\"page_bytes\": %zu, \"dirty\": {",
         (unsigned long long)m, (unsigned long long)(2 * k), ms(t0, t1), ms(t1, t2), ms(t2, t3),
         Mirror<uint8_t>::kPageBytes);
  size_t total = 0;
  const char* sep = "";
#define SHOW(a)                                                                                     \
  {                                                                                                 \
    const size_t pg = dirty_pages(ix.a);                                                            \
    const size_t b = pg * ix.a.per_page() * sizeof(ix.a.h[0]);                                      \
    total += b;                                                                                     \
    printf("%s\"%s\": {\"pages\": %zu, \"bytes\": %zu, \"all_dirty\": %d}", sep, #a, pg, b, (int)ix.a.all_dirty); \
    sep = ", ";                                                                                     \
  }
  MIRRORS(SHOW)
  printf("}, \"bytes\": %zu, \"bytes_per_op\": %.0f}\n", total, (double)total / (2 * k));
  return 0;
}

// Standalone self-test of the token-loader core (runtime/token_loader_core.h), built and run by
// tests/test_runtime_sanitizers.py under ThreadSanitizer and under AddressSanitizer + UBSan
// (race detection / sanitizers; host code only -- GPU sanitizers are not available
// on the MI355X pool).
//
//   token_loader_selftest <tmpdir>
//
// Writes .npy shards of several dtypes, then checks that every rank's Prefetcher reproduces the
// reference DataLoaderLite windows (dataloader.py:14-52) while the producer threads run: 4 ranks
// consumed concurrently from 4 threads, cursor save / restore mid-stream, reset, a zero-depth queue,
// and the malformed-file errors.  Exit status 0 = pass.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "token_loader_core.h"

using mamba_amd::loader::Cursor;
using mamba_amd::loader::NpyShard;
using mamba_amd::loader::Prefetcher;
using Buf = std::vector<int64_t>;

static int failures = 0;
#define CHECK(cond, ...)                                 \
  do {                                                   \
    if (!(cond)) {                                       \
      std::fprintf(stderr, "CHECK failed: %s: ", #cond); \
      std::fprintf(stderr, __VA_ARGS__);                 \
      std::fprintf(stderr, "\n");                        \
      ++failures;                                        \
    }                                                    \
  } while (0)

// token value at index i of shard s (distinct per shard, wraps inside every dtype used)
static int64_t tok(int s, int64_t i) { return (i * 7 + s * 1000 + 3) % 30000; }

static void write_npy(const std::string& path, int s, int64_t n, const char* descr, int itemsize) {
  char hdr[128];
  int hl = std::snprintf(hdr, sizeof(hdr), "{'descr': '%s', 'fortran_order': False, 'shape': (%lld,), }", descr,
                         (long long)n);
  int total = 10 + hl + 1;
  int pad = (64 - total % 64) % 64;
  std::string h(hdr, hl);
  h.append(pad, ' ');
  h.push_back('\n');
  FILE* f = std::fopen(path.c_str(), "wb");
  const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
  std::fwrite(magic, 1, 8, f);
  const unsigned short len = (unsigned short)h.size();
  std::fwrite(&len, 2, 1, f);
  std::fwrite(h.data(), 1, h.size(), f);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t v = tok(s, i);
    std::fwrite(&v, (size_t)itemsize, 1, f);  // little-endian host
  }
  std::fclose(f);
}

static Prefetcher<Buf>* make(const std::vector<std::string>& files, int64_t B, int64_t T, int64_t rank, int64_t world,
                             int64_t depth) {
  std::vector<std::shared_ptr<NpyShard>> sh;
  for (auto& f : files) sh.emplace_back(std::make_shared<NpyShard>(f));
  return new Prefetcher<Buf>(std::move(sh), B, T, rank, world, depth, [](int64_t n) { return Buf((size_t)n); },
                             [](Buf& b) { return b.data(); });
}

// the reference loader, sequential: returns the windows rank r sees
static std::vector<std::pair<int, int64_t>> reference(const std::vector<int64_t>& lens, int64_t B, int64_t T,
                                                      int64_t r, int64_t world, int count) {
  std::vector<std::pair<int, int64_t>> out;
  int s = 0;
  int64_t pos = B * T * r;
  for (int k = 0; k < count; ++k) {
    out.push_back({s, pos});
    pos += B * T * world;
    if (pos + B * T * world + 1 > lens[s]) {
      s = (s + 1) % (int)lens.size();
      pos = B * T * r;
    }
  }
  return out;
}

static void check_window(const Buf& b, int s, int64_t pos, int64_t n, const char* what) {
  for (int64_t i = 0; i < n; ++i)
    if (b[(size_t)i] != tok(s, pos + i)) {
      CHECK(false, "%s: shard %d pos %lld token %lld: got %lld want %lld", what, s, (long long)pos, (long long)i,
            (long long)b[(size_t)i], (long long)tok(s, pos + i));
      return;
    }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <tmpdir>\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const std::vector<int64_t> lens = {5003, 4099, 6007};
  const char* descr[] = {"<u2", "<i4", "<i8"};
  const int isz[] = {2, 4, 8};
  std::vector<std::string> files;
  for (int s = 0; s < 3; ++s) {
    files.push_back(dir + "/shard_" + std::to_string(s) + ".npy");
    write_npy(files.back(), s, lens[(size_t)s], descr[s], isz[s]);
  }
  const int64_t B = 4, T = 32, world = 4;
  const int count = 200;  // several rollovers through all shards

  // 4 ranks, each consumed on its own thread while its producer runs
  std::vector<std::thread> ths;
  for (int64_t r = 0; r < world; ++r)
    ths.emplace_back([&, r] {
      std::unique_ptr<Prefetcher<Buf>> p(make(files, B, T, r, world, 3));
      const auto ref = reference(lens, B, T, r, world, count);
      for (int k = 0; k < count; ++k) {
        const Cursor c = p->state();
        CHECK(c.shard == ref[(size_t)k].first && c.pos == ref[(size_t)k].second, "rank %lld step %d cursor", (long long)r, k);
        const Buf b = p->next();
        check_window(b, ref[(size_t)k].first, ref[(size_t)k].second, B * T + 1, "concurrent ranks");
      }
    });
  for (auto& t : ths) t.join();

  // cursor save / restore and reset while the producer is ahead of the consumer
  {
    std::unique_ptr<Prefetcher<Buf>> p(make(files, B, T, 1, world, 4));
    const auto ref = reference(lens, B, T, 1, world, count);
    for (int k = 0; k < 37; ++k) p->next();
    const Cursor saved = p->state();
    for (int k = 0; k < 11; ++k) p->next();
    p->set_state(saved.shard, saved.pos);
    for (int k = 37; k < 60; ++k) {
      const Buf b = p->next();
      check_window(b, ref[(size_t)k].first, ref[(size_t)k].second, B * T + 1, "restore");
    }
    p->reset();
    const Buf b = p->next();
    check_window(b, 0, B * T * 1, B * T + 1, "reset");
    // rapid restarts: the producer is stopped and joined mid-flight
    for (int k = 0; k < 50; ++k) p->set_state(k % 3, B * T * 1);
    const Buf b2 = p->next();
    check_window(b2, 49 % 3, B * T * 1, B * T + 1, "rapid restarts");
  }

  // depth <= 0 is clamped to a one-deep queue
  {
    std::unique_ptr<Prefetcher<Buf>> p(make(files, 2, 8, 0, 1, 0));
    const auto ref = reference(lens, 2, 8, 0, 1, 500);
    for (int k = 0; k < 500; ++k) {
      const Buf b = p->next();
      check_window(b, ref[(size_t)k].first, ref[(size_t)k].second, 17, "depth 0");
    }
  }

  // malformed inputs raise instead of reading out of bounds
  {
    const std::string bad = dir + "/bad.npy";
    FILE* f = std::fopen(bad.c_str(), "wb");
    std::fwrite("\x93NUMPY\x01\x00\xff\x7f{'descr'", 1, 17, f);  // header length beyond the file
    std::fclose(f);
    bool threw = false;
    try {
      NpyShard s(bad);
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw, "truncated header must throw");
    threw = false;
    try {
      std::unique_ptr<Prefetcher<Buf>> p(make(files, 64, 64, 3, 4, 2));  // first window beyond the shard
    } catch (const std::exception&) {
      threw = true;
    }
    CHECK(threw, "short shard must throw");
  }

  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("token_loader selftest: OK\n");
  return 0;
}

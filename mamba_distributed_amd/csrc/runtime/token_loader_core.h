// Torch-free core of the native token-shard loader (runtime/token_loader.cpp binds it to torch):
// memory-mapped .npy shards and a producer thread that assembles rank-strided batches ahead of the
// consumer.  Kept free of ATen so tests/test_runtime_sanitizers.py can build it standalone under
// ThreadSanitizer (the producer/consumer handshake) and AddressSanitizer + UBSan (header parsing, the
// widening gather) -- SURVEY.md §5.2.  Batch semantics: reference dataloader.py:14-52 (R7/R8).
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace mamba_amd {
namespace loader {

// ---- one read-only memory-mapped 1-D .npy array --------------------------------------------

// ---- one read-only memory-mapped 1-D .npy array --------------------------------------------
struct NpyShard {
  std::string path;
  void* map = nullptr;
  size_t map_len = 0;
  const uint8_t* data = nullptr;
  int64_t n = 0;
  int itemsize = 0;   // 1, 2, 4 or 8
  bool is_signed = false;

  explicit NpyShard(const std::string& p) : path(p) {
    int fd = ::open(p.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("TokenLoader: cannot open " + p);
    struct stat st;
    if (::fstat(fd, &st) != 0) { ::close(fd); throw std::runtime_error("TokenLoader: cannot stat " + p); }
    map_len = (size_t)st.st_size;
    map = ::mmap(nullptr, map_len, PROT_READ, MAP_SHARED, fd, 0);
    ::close(fd);
    if (map == MAP_FAILED) { map = nullptr; throw std::runtime_error("TokenLoader: mmap failed for " + p); }
    ::madvise(map, map_len, MADV_SEQUENTIAL);
    parse_header();
  }
  ~NpyShard() {
    if (map) ::munmap(map, map_len);
  }
  NpyShard(const NpyShard&) = delete;
  NpyShard& operator=(const NpyShard&) = delete;

  void parse_header() {
    const uint8_t* b = static_cast<const uint8_t*>(map);
    if (map_len < 10 || std::memcmp(b, "\x93NUMPY", 6) != 0) throw std::runtime_error("TokenLoader: not a .npy file: " + path);
    const int major = b[6];
    size_t hlen, off;
    if (major == 1) { hlen = b[8] | (b[9] << 8); off = 10; }
    else if (major == 2 || major == 3) {
      if (map_len < 12) throw std::runtime_error("TokenLoader: truncated header: " + path);
      hlen = (size_t)b[8] | ((size_t)b[9] << 8) | ((size_t)b[10] << 16) | ((size_t)b[11] << 24);
      off = 12;
    } else throw std::runtime_error("TokenLoader: unsupported .npy version in " + path);
    if (off + hlen > map_len) throw std::runtime_error("TokenLoader: truncated header: " + path);
    const std::string h(reinterpret_cast<const char*>(b + off), hlen);
    // descr: '<u2', '<i4', '<i8', '|u1', ... (little-endian or byte-sized only)
    const size_t d = h.find("'descr'");
    const size_t q0 = h.find('\'', h.find(':', d) + 1), q1 = h.find('\'', q0 + 1);
    if (d == std::string::npos || q0 == std::string::npos || q1 == std::string::npos)
      throw std::runtime_error("TokenLoader: no descr in " + path);
    const std::string descr = h.substr(q0 + 1, q1 - q0 - 1);
    if (descr.size() < 3 || (descr[0] != '<' && descr[0] != '|') || (descr[1] != 'u' && descr[1] != 'i'))
      throw std::runtime_error("TokenLoader: unsupported dtype " + descr + " in " + path);
    is_signed = descr[1] == 'i';
    itemsize = std::stoi(descr.substr(2));
    if (itemsize != 1 && itemsize != 2 && itemsize != 4 && itemsize != 8)
      throw std::runtime_error("TokenLoader: unsupported itemsize in " + path);
    if (h.find("'fortran_order': True") != std::string::npos)
      throw std::runtime_error("TokenLoader: fortran-ordered arrays unsupported: " + path);
    const size_t s = h.find("'shape'");
    const size_t p0 = h.find('(', s), p1 = h.find(')', p0);
    if (s == std::string::npos || p0 == std::string::npos || p1 == std::string::npos)
      throw std::runtime_error("TokenLoader: no shape in " + path);
    // 1-D (n,) or any shape: total element count = product of the dims
    int64_t count = 1;
    std::string dims = h.substr(p0 + 1, p1 - p0 - 1);
    size_t i = 0;
    bool any = false;
    while (i < dims.size()) {
      while (i < dims.size() && (dims[i] == ' ' || dims[i] == ',')) ++i;
      if (i >= dims.size()) break;
      size_t j = i;
      while (j < dims.size() && dims[j] >= '0' && dims[j] <= '9') ++j;
      if (j == i) throw std::runtime_error("TokenLoader: bad shape in " + path);
      count *= std::stoll(dims.substr(i, j - i));
      any = true;
      i = j;
    }
    n = any ? count : 1;
    data = b + off + hlen;
    if ((size_t)(data - b) + (size_t)n * itemsize > map_len) throw std::runtime_error("TokenLoader: truncated data: " + path);
  }

  // widen tokens [pos, pos+cnt) into out (int64)
  void gather(int64_t pos, int64_t cnt, int64_t* out) const {
    const uint8_t* p = data + (size_t)pos * itemsize;
    switch (itemsize * (is_signed ? -1 : 1)) {
      case 1: { auto s = reinterpret_cast<const uint8_t*>(p); for (int64_t i = 0; i < cnt; ++i) out[i] = s[i]; break; }
      case -1: { auto s = reinterpret_cast<const int8_t*>(p); for (int64_t i = 0; i < cnt; ++i) out[i] = s[i]; break; }
      case 2: { uint16_t v; for (int64_t i = 0; i < cnt; ++i) { std::memcpy(&v, p + 2 * i, 2); out[i] = v; } break; }
      case -2: { int16_t v; for (int64_t i = 0; i < cnt; ++i) { std::memcpy(&v, p + 2 * i, 2); out[i] = v; } break; }
      case 4: { uint32_t v; for (int64_t i = 0; i < cnt; ++i) { std::memcpy(&v, p + 4 * i, 4); out[i] = v; } break; }
      case -4: { int32_t v; for (int64_t i = 0; i < cnt; ++i) { std::memcpy(&v, p + 4 * i, 4); out[i] = v; } break; }
      default: std::memcpy(out, p, (size_t)cnt * 8); break;  // 8-byte ints: same representation
    }
  }
};


struct Cursor {
  int64_t shard, pos;
};

// Producer thread filling a bounded queue with (B*T+1)-token windows.  Buf is the buffer type (an
// at::Tensor in the extension, std::vector<int64_t> in the sanitizer test); `alloc(n)` makes one,
// `data(buf)` exposes its int64 storage.
template <class Buf>
class Prefetcher {
 public:
  using Alloc = std::function<Buf(int64_t)>;
  using Data = std::function<int64_t*(Buf&)>;

  Prefetcher(std::vector<std::shared_ptr<NpyShard>> shards, int64_t B, int64_t T, int64_t rank, int64_t world,
             int64_t depth, Alloc alloc, Data data)
      : shards_(std::move(shards)), B_(B), T_(T), rank_(rank), world_(world),
        depth_(std::max<int64_t>(1, depth)), alloc_(std::move(alloc)), data_(std::move(data)) {
    if (shards_.empty()) throw std::runtime_error("TokenLoader: no shards");
    if (B <= 0 || T <= 0 || world <= 0 || rank < 0 || rank >= world)
      throw std::runtime_error("TokenLoader: bad B/T/rank/world");
    for (auto& s : shards_)
      if (s->n < B * T * (rank + 1) + 1)
        throw std::runtime_error("TokenLoader: shard " + s->path + " is shorter than this rank's first window");
    cursor_ = {0, B * T * rank};
    start();
  }
  ~Prefetcher() { stop(); }
  Prefetcher(const Prefetcher&) = delete;
  Prefetcher& operator=(const Prefetcher&) = delete;

  // next window (B*T+1 tokens): blocks until the producer has one
  Buf next() {
    Item it;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return !queue_.empty() || !error_.empty(); });
      if (queue_.empty()) throw std::runtime_error("TokenLoader producer failed: " + error_);
      it = std::move(queue_.front());
      queue_.pop_front();
      cursor_ = it.after;
    }
    cv_.notify_all();
    return std::move(it.buf);
  }

  // consumer cursor: (shard, position) of the window next() returns next
  Cursor state() {
    std::lock_guard<std::mutex> lk(mu_);
    return cursor_;
  }

  void set_state(int64_t shard, int64_t pos) {
    if (shard < 0 || shard >= (int64_t)shards_.size()) throw std::runtime_error("TokenLoader: bad shard index");
    if (pos < 0 || pos + B_ * T_ + 1 > shards_[shard]->n) throw std::runtime_error("TokenLoader: position out of range");
    stop();
    {
      std::lock_guard<std::mutex> lk(mu_);
      cursor_ = {shard, pos};
    }
    start();
  }

  void reset() { set_state(0, B_ * T_ * rank_); }

  // the reference's rollover rule: next window start, or the next shard when it would overflow
  Cursor advance(Cursor c) const {
    const int64_t step = B_ * T_ * world_;
    c.pos += step;
    if (c.pos + step + 1 > shards_[c.shard]->n) {
      c.shard = (c.shard + 1) % (int64_t)shards_.size();
      c.pos = B_ * T_ * rank_;
    }
    return c;
  }

  int64_t num_shards() const { return (int64_t)shards_.size(); }
  int64_t shard_len(int64_t i) const { return shards_.at(i)->n; }

 private:
  struct Item {
    Buf buf;
    Cursor after;
  };

  void start() {
    Cursor c0;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = false;
      error_.clear();
      queue_.clear();
      c0 = cursor_;
    }
    worker_ = std::thread([this, c0] { produce(c0); });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
    std::lock_guard<std::mutex> lk(mu_);
    queue_.clear();
  }

  void produce(Cursor c) {
    try {
      while (true) {
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return stop_ || (int64_t)queue_.size() < depth_; });
          if (stop_) return;
        }
        Buf buf = alloc_(B_ * T_ + 1);
        shards_[c.shard]->gather(c.pos, B_ * T_ + 1, data_(buf));
        c = advance(c);
        {
          std::lock_guard<std::mutex> lk(mu_);
          if (stop_) return;
          queue_.push_back({std::move(buf), c});
        }
        cv_.notify_all();
      }
    } catch (const std::exception& e) {
      {
        std::lock_guard<std::mutex> lk(mu_);
        error_ = e.what();
      }
      cv_.notify_all();
    }
  }

  std::vector<std::shared_ptr<NpyShard>> shards_;
  const int64_t B_, T_, rank_, world_, depth_;
  Alloc alloc_;
  Data data_;
  Cursor cursor_{0, 0};
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Item> queue_;
  std::thread worker_;
  bool stop_ = false;
  std::string error_;
};

}  // namespace loader
}  // namespace mamba_amd

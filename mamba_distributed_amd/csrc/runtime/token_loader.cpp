// Native token-shard loader: mmap'd .npy shards + a background prefetch thread that assembles
// rank-strided (x, y) batches into (optionally pinned) host tensors ahead of the training loop.
//
// Semantics are exactly the reference's DataLoaderLite (dataloader.py:14-52):
//   * rank r starts at B*T*r inside the current shard, each batch advances by B*T*world;
//   * x = tokens[pos : pos+B*T], y = tokens[pos+1 : pos+B*T+1] (int64);
//   * when the next global window would overflow (pos + B*T*world + 1 > len) the loader moves to
//     shard (s+1) % n_shards and restarts at B*T*r.
// Differences from the reference: shards are memory-mapped instead of being
// materialised as int64 in host RAM (a 100M-token uint16 shard is 200 MB of page cache, not
// 800 MB of heap per rank), and batch assembly + the uint16 -> int64 widening run on a producer
// thread `depth` batches ahead, so the training loop only issues a non_blocking H2D copy.
//
// Exposed as the TorchScript class torch.classes.mamba_amd.TokenLoader (data/loader.py wraps it).
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>

#include "token_loader_core.h"

namespace mamba_amd {

struct TokenLoader : torch::CustomClassHolder {
  TokenLoader(std::vector<std::string> shards, int64_t B, int64_t T, int64_t rank, int64_t world, int64_t depth,
              bool pin)
      : B_(B), T_(T) {
    std::vector<std::shared_ptr<loader::NpyShard>> sh;
    for (auto& s : shards) sh.emplace_back(std::make_shared<loader::NpyShard>(s));
    auto opts = at::TensorOptions().dtype(at::kLong).pinned_memory(pin);
    pf_ = std::make_unique<loader::Prefetcher<at::Tensor>>(
        std::move(sh), B, T, rank, world, depth, [opts](int64_t n) { return at::empty({n}, opts); },
        [](at::Tensor& t) { return t.data_ptr<int64_t>(); });
  }

  // next (x, y) pair, int64 (B, T); pinned when requested
  std::tuple<at::Tensor, at::Tensor> next() {
    at::Tensor buf = pf_->next();
    return {buf.narrow(0, 0, B_ * T_).view({B_, T_}), buf.narrow(0, 1, B_ * T_).view({B_, T_})};
  }
  void reset() { pf_->reset(); }
  std::vector<int64_t> state() {
    const auto c = pf_->state();
    return {c.shard, c.pos};
  }
  void set_state(int64_t shard, int64_t pos) { pf_->set_state(shard, pos); }
  int64_t num_shards() const { return pf_->num_shards(); }
  int64_t shard_len(int64_t i) const { return pf_->shard_len(i); }

 private:
  const int64_t B_, T_;
  std::unique_ptr<loader::Prefetcher<at::Tensor>> pf_;
};

TORCH_LIBRARY_FRAGMENT(mamba_amd, m) {
  m.class_<TokenLoader>("TokenLoader")
      .def(torch::init<std::vector<std::string>, int64_t, int64_t, int64_t, int64_t, int64_t, bool>())
      .def("next", &TokenLoader::next)
      .def("reset", &TokenLoader::reset)
      .def("state", &TokenLoader::state)
      .def("set_state", &TokenLoader::set_state)
      .def("num_shards", &TokenLoader::num_shards)
      .def("shard_len", &TokenLoader::shard_len);
}

}  // namespace mamba_amd

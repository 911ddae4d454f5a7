// hashfrag.h — static hash-fragment router (reference: core/parameter/hashfrag.h).
//
// fragment i -> node id  i / (frag_num / num_nodes) + 1, clamped to
// [1, num_nodes] (hashfrag.h:30-46); to_node_id(key) = map[fmix64(key) %
// frag_num] (hashfrag.h:48-53); wire format {i32 num_nodes, i32 num_frags,
// u32 map[num_frags]} (hashfrag.h:55-85).  frag_num < num_nodes is rejected
// (the reference divides by zero).
#pragma once
#include <vector>

#include "buffer.h"
#include "common.h"
#include "ss/hash.h"

namespace ss {

class HashFrag {
 public:
  HashFrag() = default;
  HashFrag(int num_nodes, int frag_num) { init(num_nodes, frag_num); }

  void init(int num_nodes, int frag_num) {
    SS_CHECK_MSG(num_nodes > 0, "num_nodes must be > 0");
    SS_CHECK_MSG(frag_num >= num_nodes, "frag_num must be >= num_nodes");
    num_nodes_ = num_nodes;
    map_.assign((size_t)frag_num, 0);
    const int each = frag_num / num_nodes;
    for (int i = 0; i < frag_num; ++i) {
      int id = i / each + 1;
      map_[i] = (index_t)(id < 1 ? 1 : (id > num_nodes ? num_nodes : id));
    }
  }
  int to_node_id(uint64_t key) const {
    SS_CHECK_MSG(!map_.empty(), "map_table has not been inited");
    return (int)map_[fmix64(key) % (uint64_t)map_.size()];
  }
  int frag_of(uint64_t key) const { return (int)(fmix64(key) % (uint64_t)map_.size()); }

  void serialize(BinaryBuffer& bb) const {
    bb << (int32_t)num_nodes_ << (int32_t)map_.size();
    for (auto v : map_) bb << v;
  }
  void deserialize(BinaryBuffer& bb) {
    int32_t n = 0, f = 0;
    bb >> n >> f;
    SS_CHECK_MSG(f > 0, "bad hashfrag payload");
    num_nodes_ = n;
    map_.resize((size_t)f);
    for (auto& v : map_) bb >> v;
  }
  int num_nodes() const { return num_nodes_; }
  int num_frags() const { return (int)map_.size(); }
  const std::vector<index_t>& map_table() const { return map_; }
  bool inited() const { return !map_.empty(); }

 private:
  int num_nodes_ = 0;
  std::vector<index_t> map_;
};

}  // namespace ss

// ht_iterators.hh — forward iterator over a singly linked node list (reference:
// ht_iterators.hh). Used by the host-side node views of ht_chaining.hh / ht_nested.hh.
#pragma once

#include <cstddef>
#include <iterator>
#include <type_traits>

template <typename Tnode, bool IsConst>
class NodeIterator {
 public:
  using iterator_category = std::forward_iterator_tag;
  using value_type = Tnode;
  using difference_type = std::ptrdiff_t;
  using pointer = std::conditional_t<IsConst, const Tnode*, Tnode*>;
  using reference = std::conditional_t<IsConst, const Tnode&, Tnode&>;

  NodeIterator() = default;
  NodeIterator(pointer p) : _p(p) {}

  reference operator*() const { return *_p; }
  pointer operator->() const { return _p; }
  NodeIterator& operator++() {
    _p = _p ? _p->next() : nullptr;
    return *this;
  }
  NodeIterator operator++(int) {
    NodeIterator t = *this;
    ++*this;
    return t;
  }
  bool valid() const { return _p != nullptr; }
  friend bool operator==(const NodeIterator& a, const NodeIterator& b) { return a._p == b._p; }
  friend bool operator!=(const NodeIterator& a, const NodeIterator& b) { return a._p != b._p; }
  friend bool operator==(const NodeIterator& a, std::nullptr_t) { return a._p == nullptr; }
  friend bool operator!=(const NodeIterator& a, std::nullptr_t) { return a._p != nullptr; }

 private:
  pointer _p = nullptr;
};

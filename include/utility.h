/*
 * utility.h — the helper surface of the reference's include/utility.h, restated
 * for the drop-in (included from shared_tree.h exactly as the reference's
 * include/shared_tree.h:24 does, so code written against the reference --
 * compress.cpp's bytes_to_string, tests/test.cpp's chunks -- compiles unchanged).
 *
 *   foreach_pair    consecutive pairs, an odd last element alone      (ref :17-29)
 *   detail::hash    weighted sum of size_t-convertible arguments       (ref :35-52)
 *   from_bits/to_bits  bits <-> unsigned integers, LSB first          (ref :58-75)
 *   chunks          a range cut into consecutive chunks                (ref :81-131)
 *   iterator_pair   a range from two iterators                         (ref :137-152)
 *   variadic_min    minimum of a pack, ties keep the earlier argument  (ref :158-170)
 *   binary_write/binary_read  big-endian integer I/O of `bytes` bytes (ref :178-194)
 *   bytes_to_string B/KB/MB/... with 3 significant digits              (ref :200-213)
 *   progress_bar, spaces  console helpers                              (ref :219-235)
 *
 * Behaviour is the reference's, with one deliberate difference: a chunk's size()
 * is the number of elements it holds (the reference reports the nominal chunk
 * width for a short last chunk as well).
 */
#pragma once

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <iostream>
#include <iterator>
#include <sstream>
#include <string>
#include <string_view>
#include <tuple>
#include <type_traits>
#include <utility>

// (a, b, c, d, e) -> pair(a, b), pair(c, d), single(e).  Only begin()/end(),
// operator!= and prefix ++ are required of the range.
template <typename Range, typename PairFn, typename SingleFn>
void foreach_pair(Range&& range, PairFn pair_fn, SingleFn single_fn) {
  auto cur = range.begin();
  const auto last = range.end();
  while (cur != last) {
    auto&& first = *cur;
    ++cur;
    if (!(cur != last)) {
      single_fn(first);
      return;
    }
    pair_fn(first, *cur);
    ++cur;
  }
}

namespace detail {
// hash(a_1, ..., a_n) = sum_i (2^(n-i+1) + 1) * a_i, e.g. hash(l, r) = 5 l + 3 r
// (the weights of the reference's std::hash<node>).
template <typename... Args>
constexpr auto hash(const Args&... args) noexcept -> std::size_t {
  std::size_t sum = 0;
  std::size_t shift = sizeof...(Args);
  ((sum += ((std::size_t{1} << shift--) + 1) * static_cast<std::size_t>(args)), ...);
  return sum;
}
}  // namespace detail

// from_bits(b0, b1, ...) = b0 | b1 << 1 | ...
template <typename... Rest>
constexpr auto from_bits(bool low_bit, Rest... higher) noexcept -> unsigned long long {
  unsigned long long value = low_bit;
  unsigned shift = 1;
  ((value |= static_cast<unsigned long long>(static_cast<bool>(higher)) << shift++), ...);
  return value;
}

// to_bits(v)[i] = bit i of v
template <typename T>
constexpr auto to_bits(T value) noexcept -> std::array<bool, 8 * sizeof(T)> {
  std::array<bool, 8 * sizeof(T)> bits{};
  for (std::size_t i = 0; i < bits.size(); ++i) bits[i] = (value >> i) & 1;
  return bits;
}

namespace detail {
// [first, last) of any forward range, with its element count
template <typename It>
struct chunk_range {
  It first, last;
  std::size_t count;
  auto begin() const { return first; }
  auto end() const { return last; }
  auto size() const { return count; }
};

// Consecutive chunks of `width` elements (the last one may be shorter).  An lvalue
// range is referenced, an rvalue one is kept by value.
template <typename Range>
class chunk_view {
 public:
  chunk_view(Range range, std::size_t width) : range_{std::forward<Range>(range)}, width_{width ? width : 1} {}

  using base_iterator = decltype(std::begin(std::declval<Range&>()));

  class iterator {
   public:
    iterator(base_iterator at, base_iterator stop, std::size_t width) : at_{at}, stop_{stop}, width_{width} {}
    auto operator*() const {
      auto end = at_;
      std::size_t n = 0;
      while (n < width_ && end != stop_) ++end, ++n;
      return chunk_range<base_iterator>{at_, end, n};
    }
    auto operator++() -> iterator& {
      for (std::size_t n = 0; n < width_ && at_ != stop_; ++n) ++at_;
      return *this;
    }
    bool operator!=(const iterator& other) const { return at_ != other.at_; }
    bool operator==(const iterator& other) const { return at_ == other.at_; }

   private:
    base_iterator at_, stop_;
    std::size_t width_;
  };

  auto begin() { return iterator{std::begin(range_), std::end(range_), width_}; }
  auto end() { return iterator{std::end(range_), std::end(range_), width_}; }

 private:
  Range range_;
  std::size_t width_;
};

template <typename First, typename Last>
struct iterator_pair : std::pair<First, Last> {
  using std::pair<First, Last>::pair;
  auto begin() { return this->first; }
  auto end() { return this->second; }
  auto begin() const { return this->first; }
  auto end() const { return this->second; }
};
}  // namespace detail

template <typename Range>
auto chunks(Range&& range, std::size_t chunk_size) -> detail::chunk_view<Range> {
  return detail::chunk_view<Range>{std::forward<Range>(range), chunk_size};
}

template <typename First, typename Last>
auto iterator_pair(First begin, Last end) {
  return detail::iterator_pair<First, Last>{begin, end};
}

// Minimum by operator<; on ties the earlier argument wins.  Returns a reference to
// the chosen argument (valid for the caller's full expression).
template <typename T>
constexpr auto variadic_min(T&& only) noexcept -> decltype(auto) {
  return std::forward<T>(only);
}

template <typename A, typename B, typename... Rest>
constexpr auto variadic_min(A&& a, B&& b, Rest&&... rest) noexcept -> decltype(auto) {
  return b < a ? variadic_min(b, std::forward<Rest>(rest)...) : variadic_min(a, std::forward<Rest>(rest)...);
}

// The low `bytes` bytes of `value`, most significant first (the .dag byte order).
template <typename T, typename = std::enable_if_t<std::is_integral_v<T>>>
void binary_write(std::ostream& os, T value, std::size_t bytes = sizeof(T)) {
  const auto bits = static_cast<std::uint64_t>(value);
  char buf[8];
  const std::size_t n = bytes < sizeof(buf) ? bytes : sizeof(buf);
  for (std::size_t k = 0; k < n; ++k) buf[k] = static_cast<char>((bits >> (8 * (n - 1 - k))) & 0xffu);
  os.write(buf, static_cast<std::streamsize>(n));
}

template <typename T, typename = std::enable_if_t<std::is_integral_v<T>>>
void binary_read(std::istream& is, T& value, std::size_t bytes = sizeof(T)) {
  unsigned char buf[8] = {};
  const std::size_t n = bytes < sizeof(buf) ? bytes : sizeof(buf);
  is.read(reinterpret_cast<char*>(buf), static_cast<std::streamsize>(n));
  std::uint64_t bits = 0;
  for (std::size_t k = 0; k < n; ++k) bits = (bits << 8) | buf[k];
  value = static_cast<T>(bits);
}

// 1 Gbase -> "1 GB", 121024 -> "121 KB" (decimal units, three significant digits,
// the iostream default float format at precision 3)
template <typename T>
auto bytes_to_string(T bytes) -> std::string {
  static constexpr const char* unit[] = {"B", "KB", "MB", "GB", "TB", "PB", "EB"};
  constexpr std::size_t last_unit = sizeof(unit) / sizeof(unit[0]) - 1;
  double size = static_cast<double>(bytes);
  std::size_t u = 0;
  for (; size >= 1000.0 && u < last_unit; ++u) size /= 1000.0;
  char text[64];
  std::snprintf(text, sizeof(text), "%.3g %s", size, unit[u]);
  return text;
}

// "\r<name>: [####      ] 40%" with a 60-character bar
inline auto progress_bar(std::string_view name, unsigned current, unsigned end) -> std::string {
  constexpr unsigned width = 60;
  const double fraction = double(current) / double(end);
  const auto filled = unsigned(fraction * width);
  std::string line = "\r";
  line.append(name);
  line += ": [";
  for (unsigned i = 0; i < width; ++i) line += i < filled ? '#' : ' ';
  line += "] ";
  line += std::to_string(unsigned(fraction * 100));
  line += '%';
  return line;
}

inline auto spaces(unsigned length) -> std::string { return std::string(length, ' '); }

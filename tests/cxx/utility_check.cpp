// Prints the results of every utility.h helper on fixed inputs.  tests/test_dropin.py
// compiles it twice -- against this repository's include/utility.h and, when
// /root/reference exists, against the reference's include/utility.h -- and requires
// identical output (the drop-in restatement pinned against the original).
#include <array>
#include <cstdint>
#include <iostream>
#include <list>
#include <sstream>
#include <string>
#include <tuple>
#include <vector>

#include "utility.h"

int main() {
  // foreach_pair over even, odd, one and no elements
  for (int n : {0, 1, 2, 5, 8}) {
    std::vector<int> v(n);
    for (int i = 0; i < n; ++i) v[i] = 10 * i + 1;
    std::cout << "pairs " << n << ':';
    foreach_pair(
        v, [](int a, int b) { std::cout << " (" << a << ',' << b << ')'; },
        [](int a) { std::cout << " [" << a << ']'; });
    std::cout << '\n';
  }
  // chunks of arrays and lists, widths dividing the size or not (elements only:
  // the reference reports a short last chunk's size as the nominal width)
  auto a = std::array{1, 2, 3, 4, 5, 6, 7, 8};
  for (std::size_t w : {1u, 2u, 3u, 8u}) {
    std::cout << "chunks " << w << ':';
    for (auto chunk : chunks(a, w)) {
      std::cout << " {";
      for (auto x : chunk) std::cout << ' ' << x;
      std::cout << " }";
    }
    std::cout << '\n';
  }
  std::list<int> l{5, 4, 3, 2, 1};
  std::cout << "list chunks:";
  for (auto chunk : chunks(l, 2)) {
    std::cout << " {";
    for (auto x : chunk) std::cout << ' ' << x;
    std::cout << " }";
  }
  std::cout << '\n';
  // iterator_pair
  std::cout << "range:";
  for (auto x : iterator_pair(a.begin() + 2, a.begin() + 5)) std::cout << ' ' << x;
  std::cout << '\n';
  // variadic_min: value and which argument on ties
  using T = std::tuple<int, bool, bool>;
  T t0{3, false, false}, t1{2, true, false}, t2{2, false, true}, t3{2, true, true};
  const T& m = variadic_min(t0, t1, t2, t3);
  std::cout << "min " << std::get<0>(m) << std::get<1>(m) << std::get<2>(m) << ' ' << (&m == &t2) << '\n';
  int i0 = 7, i1 = 7, i2 = 9;
  std::cout << "tie " << (&variadic_min(i0, i1, i2) == &i0) << ' ' << variadic_min(5) << ' ' << variadic_min(4, 1, 3) << '\n';
  // detail::hash, from_bits, to_bits
  std::cout << "hash " << detail::hash(std::size_t{7}, std::size_t{11}) << ' ' << detail::hash(std::size_t{1}, std::size_t{2}, std::size_t{3})
            << ' ' << detail::hash(std::size_t{42}) << '\n';
  std::cout << "from_bits " << from_bits(true) << ' ' << from_bits(false, true) << ' ' << from_bits(true, false, true, true) << '\n';
  std::cout << "to_bits";
  for (bool b : to_bits(std::uint8_t{0xa5})) std::cout << b;
  std::cout << ' ';
  for (bool b : to_bits(0x80000001u)) std::cout << b;
  std::cout << '\n';
  // binary_write / binary_read: big-endian, truncated widths, round trips
  std::ostringstream os;
  binary_write(os, std::uint64_t{0x0102030405060708ull});
  binary_write(os, std::uint32_t{0xdeadbeefu}, 3);
  binary_write(os, 0x1234, 2);
  binary_write(os, std::size_t{300});
  const std::string bytes = os.str();
  std::cout << "write";
  for (unsigned char c : bytes) std::cout << ' ' << unsigned(c);
  std::cout << '\n';
  std::istringstream is(bytes);
  std::uint64_t r64 = 0;
  std::uint32_t r24 = 0;
  int r16 = 0;
  std::size_t rs = 0;
  binary_read(is, r64);
  binary_read(is, r24, 3);
  binary_read(is, r16, 2);
  binary_read(is, rs);
  std::cout << "read " << r64 << ' ' << r24 << ' ' << r16 << ' ' << rs << '\n';
  // bytes_to_string across units, rounding edges and integer types
  for (unsigned long long n : {0ull, 1ull, 999ull, 1000ull, 1023ull, 121024ull, 229354ull, 1279056ull, 999499ull,
                               999500ull, 999999ull, 1000000000ull, 3200000000ull, 123456789012345ull,
                               18446744073709551615ull})
    std::cout << "bytes " << n << " = " << bytes_to_string(n) << '\n';
  std::cout << "bytes int " << bytes_to_string(104990) << " double " << bytes_to_string(1234.5) << '\n';
  // progress_bar and spaces
  std::cout << progress_bar("Sorting nodes", 0, 1) << '|' << progress_bar("Combining subtrees", 7, 9) << '|'
            << progress_bar("x", 3, 3) << '|' << spaces(4) << "|\n";
  return 0;
}

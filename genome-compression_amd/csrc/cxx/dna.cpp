// dna value type (include/dna.h).  Restates reference src/dna.cpp:
// to_nac :25-49, random :92-96, transposed :104-111, mirrored :116-121,
// canonical :135-143, serialize/deserialize :149-161, code/nucleotide/set :167-197.
#include "dna.h"

#include <cctype>
#include <cstdlib>
#include <iostream>

namespace {

constexpr char kSymbols[16] = {'S', 'A', 'C', 'R', 'G', 'B', 'N', 'K', 'T', 'W', 'V', 'D', 'Y', 'H', 'M', '-'};

int to_code(char nucleotide) {
  const int c = std::toupper(static_cast<unsigned char>(nucleotide));
  for (int k = 0; k < 16; ++k)
    if (kSymbols[k] == c) return k;
  std::cerr << "Encountered unknown symbol: " << c << " (ASCII code " << c << ")\n";
  std::exit(1);
}

}  // namespace

dna::dna(std::string_view strand) : nucleotides{0} {
  for (std::size_t i = 0; i < length && i < strand.size(); ++i)
    nucleotides |= std::uint64_t(to_code(strand[i])) << (4 * i);
}

auto dna::random(unsigned seed) -> dna {
  std::srand(seed);
  const auto value = static_cast<unsigned long long>(std::rand() | (std::uint64_t(std::rand()) << 32));
  const auto mask = (1u << dna::size()) - 1;
  return dna{value & mask};
}

auto dna::transposed() const noexcept -> dna {
  auto v = nucleotides;
  v = ((v >> 1) & 0x5555555555555555ull) | ((v & 0x5555555555555555ull) << 1);
  v = ((v >> 2) & 0x3333333333333333ull) | ((v & 0x3333333333333333ull) << 2);
  return dna{v};
}

auto dna::mirrored() const noexcept -> dna {
  std::uint64_t r = 0;
  for (std::size_t i = 0; i < length; ++i) r |= ((nucleotides >> (4 * (length - 1 - i))) & 0xfull) << (4 * i);
  return dna{r};
}

auto dna::canonical() const noexcept -> std::tuple<dna, bool, bool, bool> {
  const bool inv = invariant();
  // lexicographic minimum of (value, m, t) over current, transposed, mirrored, inverted
  std::tuple<dna, bool, bool, bool> best{*this, false, false, inv};
  const std::tuple<dna, bool, bool, bool> cand[3] = {
      {transposed(), false, true, inv}, {mirrored(), true, false, inv}, {inverted(), true, true, inv}};
  for (const auto& c : cand)
    if (c < best) best = c;
  return best;
}

void dna::serialize(std::ostream& os) const {
  for (int i = int(bytes()) - 1; i >= 0; --i) os.put(char((nucleotides >> (8 * i)) & 0xff));
}

auto dna::deserialize(std::istream& is) -> dna {
  std::uint64_t v = 0;
  for (std::size_t i = 0; i < bytes(); ++i) v = (v << 8) | std::uint64_t(static_cast<unsigned char>(is.get()));
  return dna{v};
}

auto dna::code(std::size_t index) const -> nac { return static_cast<nac>((nucleotides >> (4 * index)) & 0xf); }

auto dna::nucleotide(std::size_t index) const -> char { return kSymbols[static_cast<int>(code(index))]; }

auto operator<<(std::ostream& os, const dna& strand) -> std::ostream& {
  for (std::size_t i = 0; i < dna::size(); ++i) os << strand.nucleotide(i);
  return os;
}

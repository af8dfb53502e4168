// fasta_reader (include/fasta_reader.h): reference src/fasta_reader.cpp:13-123.
// The file is read once; the line contract is libgcz's gcz_fasta_extract.
#include "fasta_reader.h"

#include <cstdlib>
#include <fstream>
#include <iostream>

#include "gcz.h"

fasta_reader::fasta_reader(std::filesystem::path path, std::size_t buffer_size)
    : file_path{std::move(path)}, buffer_size{buffer_size ? buffer_size : 1} {
  std::ifstream f(file_path, std::ios::binary);
  if (!f.is_open()) {   // fasta_reader.cpp:15-18
    std::cerr << "Unable to open file, aborting...\n";
    std::exit(1);
  }
  f.seekg(0, std::ios::end);
  bytes.resize(std::size_t(f.tellg()));
  f.seekg(0, std::ios::beg);
  if (!bytes.empty()) f.read(reinterpret_cast<char*>(bytes.data()), std::streamsize(bytes.size()));
  seq.resize(bytes.size());
  seq.resize(gcz_fasta_extract(bytes.data(), bytes.size(), seq.data()));
  strands = seq.size() / dna::size();
}

auto fasta_reader::read_into(std::vector<dna>& vector) -> bool {
  if (next >= strands) return false;
  const std::size_t n = std::min(buffer_size, strands - next);
  const std::size_t L = dna::size();
  vector.resize(n);
  for (std::size_t i = 0; i < n; ++i)
    vector[i] = dna{std::string_view{reinterpret_cast<const char*>(&seq[(next + i) * L]), L}};
  next += n;
  return true;
}

auto fasta_reader::size() const -> std::size_t { return bytes.size(); }

auto fasta_reader::buffers() const -> std::size_t { return size() / (buffer_size * dna::size()); }

auto read_genome(const std::filesystem::path path) -> std::vector<dna> {
  if (!std::filesystem::is_regular_file(path)) {   // fasta_reader.cpp:109-112
    std::cerr << "Non-existent path, aborting...\n";
    std::exit(1);
  }
  std::vector<dna> result, buffer;
  fasta_reader file{path};
  while (file.read_into(buffer)) result.insert(result.end(), buffer.begin(), buffer.end());
  return result;
}

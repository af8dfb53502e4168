// fasta_reader (include/fasta_reader.h): reference src/fasta_reader.cpp:13-123.
// The file is read once; the line contract is libgcz's gcz_fasta_extract.
#include "fasta_reader.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <iostream>

#include "gcz.h"

fasta_reader::fasta_reader(std::filesystem::path path, std::size_t buffer_size)
    : file_path{std::move(path)}, buffer_size{buffer_size ? buffer_size : 1} {
  const int fd = ::open(file_path.c_str(), O_RDONLY);
  struct stat st {};
  if (fd < 0 || ::fstat(fd, &st) != 0) {   // fasta_reader.cpp:15-18
    std::cerr << "Unable to open file, aborting...\n";
    std::exit(1);
  }
  nbytes = std::size_t(st.st_size);
  if (nbytes) {
    void* m = ::mmap(nullptr, nbytes, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    if (m == MAP_FAILED) {
      std::cerr << "Unable to open file, aborting...\n";
      std::exit(1);
    }
    const std::size_t n = nbytes;
    bytes = std::shared_ptr<const std::uint8_t>(static_cast<const std::uint8_t*>(m),
                                                [n](const std::uint8_t* q) { ::munmap(const_cast<std::uint8_t*>(q), n); });
  }
  ::close(fd);
}

void fasta_reader::extract() const {
  if (extracted) return;
  seq.resize(nbytes);
  seq.resize(gcz_fasta_extract(bytes.get(), nbytes, int(dna::size()), buffer_size, seq.data()));
  strands = seq.size() / dna::size();
  extracted = true;
}

auto fasta_reader::bases() const -> const std::vector<std::uint8_t>& {
  extract();
  return seq;
}

auto fasta_reader::eof() const -> bool {
  extract();
  return next >= strands && !loaded;
}

// the next buffer of strands into the back buffer (empty at the end of the file)
void fasta_reader::load_buffer() {
  extract();
  const std::size_t n = next < strands ? std::min(buffer_size, strands - next) : 0;
  const std::size_t L = dna::size();
  back.resize(n);
  for (std::size_t i = 0; i < n; ++i)
    back[i] = dna{std::string_view{reinterpret_cast<const char*>(&seq[(next + i) * L]), L}};
  next += n;
  loaded = n != 0;
}

void fasta_reader::swap_buffers() {
  std::swap(back, front);
  loaded = !back.empty();
}

auto fasta_reader::read_into(std::vector<dna>& vector) -> bool {   // src/fasta_reader.cpp:92-106
  if (!loaded) load_buffer();
  if (!loaded) return false;
  std::swap(back, vector);
  back.clear();
  loaded = false;
  return !vector.empty();
}

auto fasta_reader::size() const -> std::size_t { return nbytes; }

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

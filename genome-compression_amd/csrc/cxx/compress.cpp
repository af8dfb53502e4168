// compress — drop-in for the reference CLI (compress.cpp), backed by the
// MI355X build.  Same flags, messages, exit codes, report and --statistics
// CSV (dna_size,width,ratio,original,compressed,t_build_ms,t_sort_ms,t_total_ms;
// compress.cpp:71-79); the .dag output is byte-identical to the reference's.
// GPU selection: GCZ_DEVICE (default 0); --gpus=N spreads the build over N GPUs
// (shared_tree_on_gpus, include/shared_tree.h).
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdlib>
#include <filesystem>
#include <iostream>
#include <sstream>
#include <string_view>
#include <tuple>

#include "dna.h"
#include "fasta_reader.h"
#include "shared_tree.h"

namespace {

void print_input(const std::filesystem::path& input, std::uintmax_t file_size) {
  std::cout << "\n============================================================\n"
            << " Input\n"
            << "============================================================\n"
            << " Filename:                  " << input << '\n'
            << " Size:                      " << bytes_to_string(double(file_size)) << '\n'
            << " Nucleotides (upper bound): " << file_size << "\n\n";
}

void print_output(const std::filesystem::path& output, const std::filesystem::path& histogram,
                  std::size_t compressed_size, std::size_t width, std::size_t file_size) {
  std::cout << "\n============================================================\n"
            << " Output\n"
            << "============================================================\n";
  if (!output.empty()) std::cout << " Filename:                  " << output << '\n';
  std::cout << " Size:                      " << bytes_to_string(double(compressed_size)) << '\n'
            << " Nucleotides:               " << width * dna::size() << '\n'
            << " Compression ratio:         " << double(file_size) / double(compressed_size) << '\n';
  if (!histogram.empty()) std::cout << " Histogram:                 " << histogram << '\n';
}

void print_tree_dimensions(const shared_tree& tree, std::size_t width) {
  std::cout << "\n============================================================\n"
            << " Tree dimensions\n"
            << "============================================================\n"
            << " Leaf size:                 " << dna::size() << " nucleotides\n"
            << " Width:                     " << width << '\n'
            << " Depth:                     " << tree.depth() << '\n'
            << " Leaves:                    " << tree.leaf_count() << '\n'
            << " Nodes:                     " << tree.node_count() << '\n';
}

void print_timings(std::chrono::milliseconds construction, std::chrono::milliseconds sorting) {
  std::cout << "\n============================================================\n"
            << " Timings\n"
            << "============================================================\n"
            << " Tree construction:         " << construction.count() << " ms\n"
            << " Frequency sorting:         " << sorting.count() << " ms\n\n";
}

void print_statistics(std::size_t original, std::size_t compressed, std::size_t width,
                      std::chrono::milliseconds construction, std::chrono::milliseconds sorting) {
  std::cout << dna::size() << ',' << width << ',' << double(original) / double(compressed) << ',' << original << ','
            << compressed << ',' << construction.count() << ',' << sorting.count() << ','
            << construction.count() + sorting.count() << '\n';
}

void print_help() {
  std::cout << "Usage: compress [options] file...\n"
            << "Options:\n"
            << "\t--help\t\t\tPrints this documentation\n"
            << "\t--verbose\t\tPrint verbose output\n"
            << "\t--statistics\t\tPrint only numerical summary of output\n"
            << "\t--no-save\t\tDo not save the compressed file\n"
            << "\t--output=<file>\t\tWrite output to <file>, default being <input>.dag\n"
            << "\t--histogram=<file>\tSave histogram of node references in tree to <file>\n"
            << "\t--dna-size=<size>\tThe number of nucleotides stored per leaf node, default is 12\n"
            << "\t--gpus=<n>\t\tBuild on n GPUs (GCZ_DEVICE onwards), default is 1\n";
}

auto parse_commands(int argc, char* argv[]) {   // compress.cpp:95-165
  std::filesystem::path input, output, histogram;
  bool verbose = false, statistics = false, save = true;
  std::size_t dna_size = 12;
  int gpus = 1;
  if (argc == 1) {
    std::cout << "Invalid command: argument <file> required.\n";
    std::cout << "Use --help for more information\n";
    std::exit(2);
  }
  for (int i = 1; i < argc; ++i) {
    std::string_view a{argv[i]};
    if (a == "--help") {
      print_help();
      std::exit(0);
    } else if (a == "--verbose") {
      verbose = true;
    } else if (a == "--statistics") {
      statistics = true;
    } else if (a.substr(0, 9) == "--output=") {
      output = a.substr(9);
    } else if (a.substr(0, 12) == "--histogram=") {
      histogram = a.substr(12);
    } else if (a == "--no-save") {
      save = false;
    } else if (a.substr(0, 7) == "--gpus=") {
      gpus = std::max(1, std::atoi(std::string(a.substr(7)).c_str()));
    } else if (a.substr(0, 11) == "--dna-size=") {
      a.remove_prefix(11);
      std::cout << a << '\n';
      dna_size = std::size_t(std::atoi(a.data()));
    } else {
      if (!input.empty()) {
        std::cout << "Compression of multiple files at once is currently not supported.\n";
        std::exit(1);
      }
      input = a;
    }
  }
  if (verbose && statistics) {
    std::cout << "Invalid flag combination: --verbose and --statistics are mutually exclusive\n";
    std::cout << "Use --help for more information\n";
    std::exit(2);
  }
  if (input.empty()) {
    std::cout << "Invalid command: argument <file> required.\n";
    std::cout << "Use --help for more information\n";
    std::exit(2);
  }
  if (output.empty() && save) {
    output = input;
    output.replace_extension(".dag");
  }
  return std::tuple{input, output, histogram, verbose, statistics, dna_size, gpus};
}

}  // namespace

int main(int argc, char* argv[]) {
  auto [input, output, histogram, verbose, statistics, dna_size, gpus] = parse_commands(argc, argv);
  dna::size(dna_size);
  if (!std::filesystem::is_regular_file(input)) {
    std::cout << "Invalid filename: " << input << '\n';
    std::exit(2);
  }
  const auto original_size = std::filesystem::file_size(input);
  if (verbose) print_input(input, original_size);

  auto start = std::chrono::high_resolution_clock::now();
  auto compressed = gpus > 1 ? shared_tree_on_gpus(input, gpus) : shared_tree{input};
  auto end = std::chrono::high_resolution_clock::now();
  const auto construction = std::chrono::duration_cast<std::chrono::milliseconds>(end - start);

  start = std::chrono::high_resolution_clock::now();
  compressed.sort_tree(verbose);
  end = std::chrono::high_resolution_clock::now();
  const auto sorting = std::chrono::duration_cast<std::chrono::milliseconds>(end - start);

  const auto compressed_size = compressed.bytes();
  const auto width = compressed.width();
  if (!histogram.empty()) compressed.store_histogram(histogram);
  if (!output.empty()) compressed.save(output);
  if (verbose) {
    print_output(output, histogram, compressed_size, width, original_size);
    print_tree_dimensions(compressed, width);
    print_timings(construction, sorting);
  }
  if (statistics) print_statistics(original_size, compressed_size, width, construction, sorting);
  return 0;
}

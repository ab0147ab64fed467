// xflow-amd: libffm block reader.
//
// Behaviour of the reference's only live loader,
// LoadData::load_minibatch_hash_data_fread (/root/reference/src/io/
// load_data_from_disk.cc:103-210):
//   * a block is up to block_size-1 bytes; when the buffer fills, it is cut at
//     the last '\n' and the remainder carries over to the next block;
//   * a row is `label<TAB>fgid:fid:val fgid:fid:val ...`; label = atof > 1e-7;
//   * fgid = atof(text before the first ':'), key = std::hash<std::string> of
//     the text between the first and second ':'; the value is NOT parsed;
//   * CRLF line ends are harmless (the '\r' lands in the ignored value).
// Deliberate, documented deviations on malformed input (the reference reads
// out of bounds there): lines without a TAB are skipped, empty tokens are
// skipped, and a 2-part token `a:b` yields fgid=atof(a), fid=hash(b).
//
// Two APIs are provided: the reference-compatible LoadData / Data / kv
// (io.h:18-65, load_data_from_disk.h:19-34) and a CSR block reader used by the
// GPU pipeline (row_ptr / keys / fgid / labels in flat arrays), with an
// optional background prefetch thread that parses block i+1 while block i
// trains.
#pragma once

#include <cstdio>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace xflow {

// ---- reference-compatible data structures (io.h:18-22, :61-65) ----
struct kv {
  int fgid;
  size_t fid;
  int val;
};

class Data {
 public:
  std::vector<std::vector<kv>> fea_matrix;
  std::vector<int> label;
};

// ---- CSR block ----
struct CsrBlock {
  std::vector<int32_t> row_ptr{0};
  std::vector<uint64_t> keys;
  std::vector<int32_t> fgid;
  std::vector<float> labels;
  int32_t max_fgid = 0;
  int64_t rows() const { return (int64_t)labels.size(); }
  int64_t nnz() const { return (int64_t)keys.size(); }
  void clear() {
    row_ptr.assign(1, 0);
    keys.clear();
    fgid.clear();
    labels.clear();
    max_fgid = 0;
  }
};

// std::hash<std::string> of the feature text (libstdc++ _Hash_bytes, seed
// 0xc70f6907) -- identical keys to the reference.
uint64_t feature_hash(const char* p, size_t n);

// Parse a NUL-free text range holding whole lines into `out` (appends).
void parse_libffm(const char* text, size_t n, CsrBlock& out);
// The same with the range split at line boundaries over `threads` threads
// (segments of >= 256 KB); the result is identical to parse_libffm.
void parse_libffm_parallel(const char* text, size_t n, CsrBlock& out, int threads);
int default_parse_threads();  // min(hardware_concurrency, 16)

class BlockReader {
 public:
  BlockReader(const std::string& path, size_t block_bytes);
  ~BlockReader();
  BlockReader(const BlockReader&) = delete;
  BlockReader& operator=(const BlockReader&) = delete;
  // Next block; returns false (and an empty block) at end of file.
  bool next(CsrBlock& out);
  void rewind();
  const std::string& path() const { return path_; }
  // threads used to parse one block (1 = serial, the reference's LoadData)
  void set_parse_threads(int t) { parse_threads_ = t < 1 ? 1 : t; }
  int parse_threads() const { return parse_threads_; }

 private:
  size_t fill_block(const char** text);  // returns length of the block's text
  int parse_threads_ = default_parse_threads();
  std::string path_;
  FILE* fp_ = nullptr;
  std::vector<char> buf_;
  size_t btop_ = 0, bmax_ = 0;
};

// Background-thread prefetching wrapper: parses the next block while the
// caller consumes the current one.
class PrefetchReader {
 public:
  PrefetchReader(const std::string& path, size_t block_bytes);
  ~PrefetchReader();
  bool next(CsrBlock& out);

 private:
  void run();
  BlockReader reader_;
  std::thread th_;
  std::mutex mu_;
  std::condition_variable cv_;
  CsrBlock slot_;
  bool full_ = false, eof_ = false, stop_ = false;
};

// ---- reference-compatible IO base (io.h:24-59) ----
// Opening a missing file throws std::runtime_error (the reference exit(1)s).
class IO {
 public:
  explicit IO(const char* file_path);
  virtual ~IO();
  void Init();
  virtual void load_all_data() = 0;
  virtual void load_minibatch_data(int num) = 0;
  const char* file_path;

 protected:
  bool next_line(std::string& line);  // false at EOF
  FILE* fp_ = nullptr;
};

// ---- reference-compatible loader (load_data_from_disk.h:19-34) ----
// load_minibatch_hash_data_fread is the reference's live loader (block read,
// libffm, hashed fid).  The other four are the reference's unused loaders,
// implemented with their intended semantics:
//   load_all_data / load_minibatch_data(num): numeric `fgid:fid:val` triples
//     (fid used as the key verbatim, val kept), whole file / next num lines;
//   load_all_hash_data / load_mibibatch_hash_data(num) [sic]: every
//     whitespace token hashed whole (sscanf("%s") + std::hash in the
//     reference), fgid = 0.
class LoadData : public IO {
 public:
  LoadData(const char* file_path, size_t block_size);
  ~LoadData() override;
  void load_all_data() override;
  void load_minibatch_data(int num) override;
  void load_all_hash_data();
  void load_mibibatch_hash_data(int num);
  void load_minibatch_hash_data_fread();
  Data m_data;

 private:
  void parse_numeric_line(const std::string& line);
  void parse_hashed_line(const std::string& line);
  std::unique_ptr<BlockReader> reader_;
  CsrBlock block_;
};

}  // namespace xflow

#pragma once
#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace dtf {

class RecordWriter {
 public:
  explicit RecordWriter(const std::string& path, bool append = false);
  ~RecordWriter();
  void write(const std::string& data);
  void flush();
  void close();
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  FILE* f_ = nullptr;
};

class RecordReader {
 public:
  explicit RecordReader(const std::string& path);
  ~RecordReader();
  bool next(std::string* out);

 private:
  std::string path_;
  FILE* f_ = nullptr;
};

struct ParsedEvent {
  double wall_time = 0;
  int64_t step = 0;
  std::string file_version;
  std::vector<std::pair<std::string, float>> scalars;
  std::vector<std::pair<std::string, std::pair<double, double>>> histograms;  // tag -> (num, sum)
};

std::string encode_scalar_event(double wall_time, int64_t step,
                                const std::vector<std::pair<std::string, float>>& kv);
std::string encode_histogram_event(double wall_time, int64_t step, const std::string& tag,
                                   const std::vector<double>& values, int nbuckets);
ParsedEvent parse_event(const std::string& data);

class EventsWriter {
 public:
  EventsWriter(const std::string& prefix, const std::string& suffix = "");
  void write_event(const std::string& serialized);
  void flush();
  void close();
  const std::string& path() const { return path_; }

 private:
  std::string path_;
  std::unique_ptr<RecordWriter> w_;
};

}  // namespace dtf

// TensorFlow tensor-bundle (Saver V2 checkpoint) codec -- SURVEY §2.7, §5.4, Appendix A.4.
//
// A bundle is <prefix>.index + <prefix>.data-00000-of-00001. The index is a LevelDB-format table (data blocks
// with prefix-compressed keys and a restart every 16 entries, an empty metaindex block, an index block mapping the
// shortest successor of each block's last key to its BlockHandle, a 48-byte footer with magic
// 0xdb4775248b80fb57). Every block carries a trailer byte (compression = none) and the masked CRC32C of
// block||type. Key "" holds a BundleHeaderProto; every other key a BundleEntryProto (dtype, shape, shard_id,
// offset, size, masked crc32c of the tensor bytes). The data file is the raw little-endian tensors concatenated
// in key order.
//
// The writer reproduces TensorFlow's byte layout exactly (the demo checkpoint of the reference re-serialises
// byte-identically, tests/test_ckpt.py), so checkpoints written here open in TensorFlow and vice versa.
#pragma once
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace tfb {

struct Entry {
  std::string key;
  int dtype = 1;                 // TF DataType enum (1 = DT_FLOAT)
  std::vector<int64_t> shape;
  int32_t shard_id = 0;
  int64_t offset = 0;
  int64_t size = 0;
  uint32_t crc32c = 0;           // masked
  bool has_crc = true;
};

struct Header {
  int32_t num_shards = 1;
  int32_t endianness = 0;        // 0 = LITTLE
  int32_t producer = 1;
  int32_t min_consumer = 0;
};

class FormatError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

uint32_t crc32c(const uint8_t* data, size_t n, uint32_t init = 0);
uint32_t mask_crc(uint32_t crc);
uint32_t unmask_crc(uint32_t masked);

// index (table) <-> header + entries
void parse_index(const std::string& bytes, Header* header, std::vector<Entry>* entries);
std::string build_index(const Header& header, const std::vector<Entry>& entries, int restart_interval = 16,
                        size_t block_size = 262144);

// protobuf pieces
std::string encode_header(const Header& h);
std::string encode_entry(const Entry& e);
Header decode_header(const std::string& v);
Entry decode_entry(const std::string& key, const std::string& v);

// whole bundle: entries are laid out in sorted key order with contiguous offsets, crcs computed here
struct Tensor {
  std::string key;
  int dtype;
  std::vector<int64_t> shape;
  std::string data;              // raw little-endian bytes
};
void write_bundle(const std::string& prefix, std::vector<Tensor> tensors);
std::vector<Tensor> read_bundle(const std::string& prefix, bool verify_crc = true);

size_t dtype_size(int dtype);

}  // namespace tfb

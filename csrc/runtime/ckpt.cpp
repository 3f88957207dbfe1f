// Deterministic ("bit-compatible") model checkpoint writer / verifier.
//
// Reference: QDecisionPolicyActor calls saveSnapshot((session, iteration)) every
// 500 updates but the body is empty (QDecisionPolicyActor.scala:74,91-93), and
// Akka Persistence's snapshot store would Java-serialize whatever it is given.
// Here a checkpoint is a named-tensor archive whose bytes are a pure function of
// (entries in the given order, their dtype/shape/bytes, metadata string):
// identical learner state => byte-identical file, across runs and machines.
//
//   "STCKPT01" u32 version(=1) u32 n_entries u64 meta_len  meta bytes   pad->64
//   table, per entry: u16 name_len name u8 dtype u8 ndim i64 shape[ndim]
//                     u64 offset u64 nbytes u32 masked_crc32c(data)      pad->64
//   data blobs, each at a 64-byte aligned offset (zero padding)
//   trailer: u64 table_end u32 masked_crc32c(bytes [0, table_end)) "STCKEND1"
// Published atomically: write <path>.tmp, fsync, rename.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "crc32c.h"

namespace {

constexpr char kMagic[8] = {'S', 'T', 'C', 'K', 'P', 'T', '0', '1'};
constexpr char kEnd[8] = {'S', 'T', 'C', 'K', 'E', 'N', 'D', '1'};

size_t align64(size_t x) { return (x + 63) & ~size_t(63); }

template <class T>
void put(std::vector<uint8_t>& b, T v) {
  const size_t o = b.size();
  b.resize(o + sizeof(T));
  std::memcpy(&b[o], &v, sizeof(T));
}

bool write_all(int fd, const void* buf, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(buf);
  while (n) {
    ssize_t w = ::write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

}  // namespace

extern "C" {

// Write a checkpoint.  shapes is the concatenation of every entry's shape.
// Returns total bytes written, or -1.
int64_t st_ckpt_write(const char* path, int n, const char* const* names, const int* dtypes, const int* ndims,
                      const int64_t* shapes, const void* const* datas, const uint64_t* nbytes, const char* meta,
                      uint64_t meta_len, int do_fsync) {
  std::vector<uint8_t> head;
  head.insert(head.end(), kMagic, kMagic + 8);
  put<uint32_t>(head, 1u);
  put<uint32_t>(head, (uint32_t)n);
  put<uint64_t>(head, meta_len);
  head.insert(head.end(), meta, meta + meta_len);
  head.resize(align64(head.size()), 0);
  // table size is needed to place data: compute it first
  size_t table_sz = 0;
  for (int i = 0; i < n; ++i) table_sz += 2 + std::strlen(names[i]) + 1 + 1 + 8 * (size_t)ndims[i] + 8 + 8 + 4;
  size_t data_off = align64(head.size() + table_sz);
  std::vector<uint64_t> offs(n);
  for (int i = 0; i < n; ++i) {
    offs[i] = data_off;
    data_off = align64(data_off + nbytes[i]);
  }
  const int64_t* sp = shapes;
  for (int i = 0; i < n; ++i) {
    const size_t nl = std::strlen(names[i]);
    put<uint16_t>(head, (uint16_t)nl);
    head.insert(head.end(), names[i], names[i] + nl);
    put<uint8_t>(head, (uint8_t)dtypes[i]);
    put<uint8_t>(head, (uint8_t)ndims[i]);
    for (int d = 0; d < ndims[i]; ++d) put<int64_t>(head, *sp++);
    put<uint64_t>(head, offs[i]);
    put<uint64_t>(head, nbytes[i]);
    put<uint32_t>(head, strt::crc_mask(strt::crc32c(datas[i], nbytes[i])));
  }
  const uint64_t table_end = head.size();
  const uint32_t head_crc = strt::crc_mask(strt::crc32c(head.data(), head.size()));
  head.resize(n ? offs[0] : align64(head.size()), 0);

  const std::string tmp = std::string(path) + ".tmp";
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return -1;
  bool ok = write_all(fd, head.data(), head.size());
  uint64_t pos = head.size();
  static const uint8_t zeros[64] = {0};
  for (int i = 0; ok && i < n; ++i) {
    if (pos < offs[i]) {
      ok = write_all(fd, zeros, offs[i] - pos);
      pos = offs[i];
    }
    ok = ok && write_all(fd, datas[i], nbytes[i]);
    pos += nbytes[i];
    const uint64_t nxt = align64(pos);
    if (ok && i + 1 < n && nxt > pos) {
      ok = write_all(fd, zeros, nxt - pos);
      pos = nxt;
    }
  }
  std::vector<uint8_t> tail;
  put<uint64_t>(tail, table_end);
  put<uint32_t>(tail, head_crc);
  tail.insert(tail.end(), kEnd, kEnd + 8);
  ok = ok && write_all(fd, tail.data(), tail.size());
  pos += tail.size();
  if (ok && do_fsync) ok = fsync(fd) == 0;
  ::close(fd);
  if (!ok || ::rename(tmp.c_str(), path) != 0) {
    ::unlink(tmp.c_str());
    return -1;
  }
  return (int64_t)pos;
}

}  // extern "C"

// Append-only event journal + snapshot store (the engine's Akka Persistence backend).
//
// Reference: SharePriceGetter persists an `Event(stockName, prices)` after each
// query and replays the journal on restart (SharePriceGetter.scala:36-40,49-52,55-62);
// the journal is LevelDB at target/my/journal, snapshots go to the local
// store at target/my/snapshots (src/main/resources/application.conf:5-18).
//
// Journal file  <dir>/<pid>.journal :
//   header  "STJRNL01"                                     (8 B)
//   record  [u32 len][u32 masked crc32c][u64 seq][u8 type][payload: len bytes]
//           crc covers seq|type|payload; type 0 = event, 1 = delete-to marker
//           (payload = u64 seq).  Little-endian, no padding: the bytes written
//           are a pure function of the (seq, type, payload) sequence.
// Recovery scans records in order and stops at the first torn / corrupt
// record, truncating the file there (a crash mid-append loses only that record).
//
// Snapshot file <dir>/snapshot-<pid>-<seq:020>-<ts:020>.snap :
//   "STSNAP01" [u64 seq][i64 ts][u64 len][u32 masked crc][payload]
//   written to a .tmp file, fsync'ed, then renamed (atomic publish).
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "crc32c.h"

namespace strt {
namespace {

constexpr char kJournalMagic[8] = {'S', 'T', 'J', 'R', 'N', 'L', '0', '1'};
constexpr char kSnapMagic[8] = {'S', 'T', 'S', 'N', 'A', 'P', '0', '1'};
constexpr size_t kRecHeader = 4 + 4 + 8 + 1;

void put_u32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }
void put_u64(uint8_t* p, uint64_t v) { std::memcpy(p, &v, 8); }
uint32_t get_u32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
uint64_t get_u64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
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

bool read_file(const std::string& path, std::vector<uint8_t>& out) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    return false;
  }
  out.resize((size_t)st.st_size);
  size_t off = 0;
  while (off < out.size()) {
    ssize_t r = ::read(fd, out.data() + off, out.size() - off);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      break;
    }
    off += (size_t)r;
  }
  ::close(fd);
  out.resize(off);
  return true;
}

int mkdirs(const std::string& dir) {
  std::string cur;
  for (size_t i = 0; i < dir.size(); ++i) {
    cur.push_back(dir[i]);
    if (dir[i] == '/' || i + 1 == dir.size()) {
      if (cur.size() > 1 && ::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
    }
  }
  return 0;
}

uint32_t record_crc(uint64_t seq, uint8_t type, const void* payload, size_t n) {
  uint8_t h[9];
  put_u64(h, seq);
  h[8] = type;
  uint32_t c = crc32c_extend(0, h, 9);
  c = crc32c_extend(c, payload, n);
  return crc_mask(c);
}

// Exact snapshot file name "snapshot-<pid>-<seq:020>-<ts:020>.snap" (no extra characters): a plain
// prefix match would let pid "x" claim the snapshots of pid "x-1".
bool parse_snap_name(const std::string& nm, const std::string& prefix, long long* seq, long long* ts) {
  constexpr size_t kW = 20;
  if (nm.size() != prefix.size() + kW + 1 + kW + 5) return false;
  if (nm.compare(0, prefix.size(), prefix) != 0) return false;
  const char* p = nm.c_str() + prefix.size();
  for (size_t i = 0; i < kW; ++i)
    if (p[i] < '0' || p[i] > '9') return false;
  if (p[kW] != '-') return false;
  for (size_t i = 0; i < kW; ++i)
    if (p[kW + 1 + i] < '0' || p[kW + 1 + i] > '9') return false;
  if (std::memcmp(p + 2 * kW + 1, ".snap", 5) != 0) return false;
  *seq = std::strtoll(std::string(p, kW).c_str(), nullptr, 10);
  *ts = std::strtoll(std::string(p + kW + 1, kW).c_str(), nullptr, 10);
  return true;
}

struct Record {
  uint64_t seq;
  uint8_t type;
  size_t off;  // payload offset in the file image
  uint32_t len;
};

}  // namespace

struct Journal {
  std::string path;
  int fd = -1;
  int fsync_mode = 0;  // 0 = none, 1 = fdatasync every append
  uint64_t highest = 0;
  uint64_t deleted_to = 0;
  uint64_t truncated_bytes = 0;
  std::mutex mu;
};

}  // namespace strt

using strt::Journal;

extern "C" {

// Open (or create) <dir>/<pid>.journal.  Returns nullptr on error (errno set).
void* st_journal_open(const char* dir, const char* pid, int fsync_mode) {
  using namespace strt;
  if (mkdirs(dir) != 0) return nullptr;
  auto* j = new Journal();
  j->path = std::string(dir) + "/" + pid + ".journal";
  j->fsync_mode = fsync_mode;
  std::vector<uint8_t> img;
  bool exists = read_file(j->path, img);
  size_t good = 0;
  if (exists && img.size() >= 8 && std::memcmp(img.data(), kJournalMagic, 8) == 0) {
    size_t off = 8;
    good = 8;
    while (off + kRecHeader <= img.size()) {
      const uint32_t len = get_u32(&img[off]);
      const uint32_t crc = get_u32(&img[off + 4]);
      const uint64_t seq = get_u64(&img[off + 8]);
      const uint8_t type = img[off + 16];
      if (off + kRecHeader + len > img.size()) break;
      if (record_crc(seq, type, &img[off + kRecHeader], len) != crc) break;
      if (seq != j->highest + 1 && type == 0) break;
      if (type == 0) j->highest = seq;
      if (type == 1 && len == 8) {
        const uint64_t d = get_u64(&img[off + kRecHeader]);
        if (d > j->deleted_to) j->deleted_to = d;
      }
      off += kRecHeader + len;
      good = off;
    }
  }
  j->fd = ::open(j->path.c_str(), O_RDWR | O_CREAT, 0644);
  if (j->fd < 0) {
    delete j;
    return nullptr;
  }
  if (good == 0) {
    if (ftruncate(j->fd, 0) != 0 || !write_all(j->fd, kJournalMagic, 8)) {
      ::close(j->fd);
      delete j;
      return nullptr;
    }
    good = 8;
  } else if (good < img.size()) {
    j->truncated_bytes = img.size() - good;
    if (ftruncate(j->fd, (off_t)good) != 0) {
      ::close(j->fd);
      delete j;
      return nullptr;
    }
  }
  ::lseek(j->fd, (off_t)good, SEEK_SET);
  return j;
}

// Write one framed buffer at the journal's end.  A failed write (e.g. ENOSPC part-way) is rolled
// back -- the file is truncated to the offset before the append and the position reset -- so a later
// successful append is never written behind a torn record (which recovery would truncate away).
static bool write_or_rollback(Journal* j, const void* buf, size_t n) {
  using namespace strt;
  const off_t at = ::lseek(j->fd, 0, SEEK_CUR);
  if (at < 0) return false;
  if (write_all(j->fd, buf, n) && (j->fsync_mode != 1 || fdatasync(j->fd) == 0)) return true;
  const int saved = errno;
  if (ftruncate(j->fd, at) == 0) ::lseek(j->fd, at, SEEK_SET);
  errno = saved;
  return false;
}

static int64_t append_record(Journal* j, uint8_t type, uint64_t seq, const void* payload, size_t n) {
  using namespace strt;
  std::vector<uint8_t> buf(kRecHeader + n);
  put_u32(&buf[0], (uint32_t)n);
  put_u32(&buf[4], record_crc(seq, type, payload, n));
  put_u64(&buf[8], seq);
  buf[16] = type;
  if (n) std::memcpy(&buf[kRecHeader], payload, n);
  if (!write_or_rollback(j, buf.data(), buf.size())) return -1;
  return (int64_t)seq;
}

// Append one event; returns its sequence number (1-based) or -1.
int64_t st_journal_append(void* h, const void* payload, size_t n) {
  auto* j = static_cast<Journal*>(h);
  std::lock_guard<std::mutex> g(j->mu);
  const int64_t r = append_record(j, 0, j->highest + 1, payload, n);
  if (r > 0) j->highest = (uint64_t)r;
  return r;
}

// Atomic batch append (persistAll): one write() for all events.
int64_t st_journal_append_batch(void* h, int count, const void* const* payloads, const size_t* sizes) {
  using namespace strt;
  auto* j = static_cast<Journal*>(h);
  std::lock_guard<std::mutex> g(j->mu);
  std::vector<uint8_t> buf;
  uint64_t seq = j->highest;
  for (int i = 0; i < count; ++i) {
    const size_t n = sizes[i];
    const size_t o = buf.size();
    buf.resize(o + kRecHeader + n);
    ++seq;
    put_u32(&buf[o], (uint32_t)n);
    put_u32(&buf[o + 4], record_crc(seq, 0, payloads[i], n));
    put_u64(&buf[o + 8], seq);
    buf[o + 16] = 0;
    if (n) std::memcpy(&buf[o + kRecHeader], payloads[i], n);
  }
  if (!write_or_rollback(j, buf.data(), buf.size())) return -1;
  j->highest = seq;
  return (int64_t)seq;
}

int64_t st_journal_highest(void* h) { return (int64_t) static_cast<Journal*>(h)->highest; }
int64_t st_journal_deleted_to(void* h) { return (int64_t) static_cast<Journal*>(h)->deleted_to; }
int64_t st_journal_truncated_bytes(void* h) { return (int64_t) static_cast<Journal*>(h)->truncated_bytes; }

// Logical deletion of events <= seq (deleteMessages(toSequenceNr)).
int st_journal_delete_to(void* h, int64_t seq) {
  using namespace strt;
  auto* j = static_cast<Journal*>(h);
  std::lock_guard<std::mutex> g(j->mu);
  uint8_t p[8];
  put_u64(p, (uint64_t)seq);
  if (append_record(j, 1, j->highest, p, 8) < 0) return -1;
  if ((uint64_t)seq > j->deleted_to) j->deleted_to = (uint64_t)seq;
  return 0;
}

typedef int (*st_replay_cb)(int64_t seq, const void* payload, size_t n, void* user);

// Replay events with from <= seq <= to (to < 0: all), skipping deleted ones.
// Returns the number of events delivered, or -1.
int64_t st_journal_replay(void* h, int64_t from, int64_t to, st_replay_cb cb, void* user) {
  using namespace strt;
  auto* j = static_cast<Journal*>(h);
  std::vector<uint8_t> img;
  {
    std::lock_guard<std::mutex> g(j->mu);
    if (!read_file(j->path, img)) return -1;
  }
  if (img.size() < 8) return 0;
  std::vector<Record> recs;
  uint64_t deleted = 0;
  size_t off = 8;
  while (off + kRecHeader <= img.size()) {
    const uint32_t len = get_u32(&img[off]);
    const uint32_t crc = get_u32(&img[off + 4]);
    const uint64_t seq = get_u64(&img[off + 8]);
    const uint8_t type = img[off + 16];
    if (off + kRecHeader + len > img.size()) break;
    if (record_crc(seq, type, &img[off + kRecHeader], len) != crc) break;
    if (type == 0) recs.push_back({seq, type, off + kRecHeader, len});
    if (type == 1 && len == 8) {
      const uint64_t d = get_u64(&img[off + kRecHeader]);
      if (d > deleted) deleted = d;
    }
    off += kRecHeader + len;
  }
  int64_t n = 0;
  for (const auto& r : recs) {
    if (r.seq <= deleted || (int64_t)r.seq < from || (to >= 0 && (int64_t)r.seq > to)) continue;
    if (cb((int64_t)r.seq, &img[r.off], r.len, user) != 0) break;
    ++n;
  }
  return n;
}

int st_journal_sync(void* h) {
  auto* j = static_cast<Journal*>(h);
  std::lock_guard<std::mutex> g(j->mu);
  return fdatasync(j->fd);
}

void st_journal_close(void* h) {
  auto* j = static_cast<Journal*>(h);
  if (!j) return;
  if (j->fd >= 0) ::close(j->fd);
  delete j;
}

// ------------------------------------------------------------------ snapshots
int st_snapshot_save(const char* dir, const char* pid, int64_t seq, int64_t ts, const void* payload, size_t n) {
  using namespace strt;
  if (mkdirs(dir) != 0) return -1;
  char name[512];
  std::snprintf(name, sizeof(name), "%s/snapshot-%s-%020lld-%020lld.snap", dir, pid, (long long)seq, (long long)ts);
  const std::string fin(name), tmp = fin + ".tmp";
  std::vector<uint8_t> buf(8 + 8 + 8 + 8 + 4 + n);
  std::memcpy(buf.data(), kSnapMagic, 8);
  put_u64(&buf[8], (uint64_t)seq);
  put_u64(&buf[16], (uint64_t)ts);
  put_u64(&buf[24], (uint64_t)n);
  put_u32(&buf[32], crc_mask(crc32c(payload, n)));
  if (n) std::memcpy(&buf[36], payload, n);
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) return -1;
  const bool ok = write_all(fd, buf.data(), buf.size()) && fsync(fd) == 0;
  ::close(fd);
  if (!ok || ::rename(tmp.c_str(), fin.c_str()) != 0) {
    ::unlink(tmp.c_str());
    return -1;
  }
  return 0;
}

// Find the newest valid snapshot with seq <= max_seq (max_seq < 0: any).
// Writes its path to path_out; returns 1 if found, 0 if none, -1 on error.
int st_snapshot_latest(const char* dir, const char* pid, int64_t max_seq, int64_t* seq_out, int64_t* ts_out,
                       char* path_out, size_t path_cap) {
  using namespace strt;
  DIR* d = opendir(dir);
  if (!d) return 0;
  const std::string prefix = std::string("snapshot-") + pid + "-";
  std::string best;
  long long best_seq = -1, best_ts = -1;
  while (dirent* e = readdir(d)) {
    std::string nm = e->d_name;
    long long s = -1, t = -1;
    if (!parse_snap_name(nm, prefix, &s, &t)) continue;
    if (max_seq >= 0 && s > max_seq) continue;
    if (s > best_seq || (s == best_seq && t > best_ts)) {
      std::vector<uint8_t> img;
      const std::string full = std::string(dir) + "/" + nm;
      if (!read_file(full, img) || img.size() < 36 || std::memcmp(img.data(), kSnapMagic, 8) != 0) continue;
      const uint64_t n = get_u64(&img[24]);
      if (36 + n != img.size() || crc_mask(crc32c(&img[36], n)) != get_u32(&img[32])) continue;
      best_seq = s;
      best_ts = t;
      best = full;
    }
  }
  closedir(d);
  if (best_seq < 0) return 0;
  *seq_out = best_seq;
  *ts_out = best_ts;
  std::snprintf(path_out, path_cap, "%s", best.c_str());
  return 1;
}

// Read a snapshot's payload (validated).  Returns payload length, or -1.
// Call with buf=nullptr to query the length.
int64_t st_snapshot_read(const char* path, void* buf, size_t cap) {
  using namespace strt;
  std::vector<uint8_t> img;
  if (!read_file(path, img) || img.size() < 36 || std::memcmp(img.data(), kSnapMagic, 8) != 0) return -1;
  const uint64_t n = get_u64(&img[24]);
  if (36 + n != img.size() || crc_mask(crc32c(&img[36], n)) != get_u32(&img[32])) return -1;
  if (buf) {
    if (cap < n) return -1;
    std::memcpy(buf, &img[36], n);
  }
  return (int64_t)n;
}

// Delete snapshots with seq <= max_seq (deleteSnapshots(criteria)).
int st_snapshot_delete_to(const char* dir, const char* pid, int64_t max_seq) {
  DIR* d = opendir(dir);
  if (!d) return 0;
  const std::string prefix = std::string("snapshot-") + pid + "-";
  int n = 0;
  std::vector<std::string> victims;
  while (dirent* e = readdir(d)) {
    std::string nm = e->d_name;
    long long s = -1, t = -1;
    if (!strt::parse_snap_name(nm, prefix, &s, &t)) continue;
    if (s <= max_seq) victims.push_back(std::string(dir) + "/" + nm);
  }
  closedir(d);
  for (auto& v : victims)
    if (::unlink(v.c_str()) == 0) ++n;
  return n;
}

}  // extern "C"

// Native self-test of the host runtime (journal, snapshot store, checkpoint writer,
// CRC32C), built standalone under AddressSanitizer+UBSan and ThreadSanitizer by
// tests/test_sanitizers.py — the race / memory-safety check of the C++ side
// (SURVEY §5.2).  Exit status 0 = pass.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

extern "C" {
uint32_t st_crc32c(const void* data, size_t n, uint32_t init);
uint32_t st_crc32c_sw(const void* data, size_t n, uint32_t init);
void* st_journal_open(const char* dir, const char* pid, int fsync_mode);
int64_t st_journal_append(void* h, const void* payload, size_t n);
int64_t st_journal_highest(void* h);
typedef int (*st_replay_cb)(int64_t seq, const void* payload, size_t n, void* user);
int64_t st_journal_replay(void* h, int64_t from, int64_t to, st_replay_cb cb, void* user);
int st_journal_delete_to(void* h, int64_t seq);
void st_journal_close(void* h);
int st_snapshot_save(const char* dir, const char* pid, int64_t seq, int64_t ts, const void* payload, size_t n);
int st_snapshot_latest(const char* dir, const char* pid, int64_t max_seq, int64_t* seq_out, int64_t* ts_out,
                       char* path_out, size_t path_cap);
int64_t st_snapshot_read(const char* path, void* buf, size_t cap);
int64_t st_ckpt_write(const char* path, int n, const char* const* names, const int* dtypes, const int* ndims,
                      const int64_t* shapes, const void* const* datas, const uint64_t* nbytes, const char* meta,
                      uint64_t meta_len, int do_fsync);
}

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

static int count_cb(int64_t seq, const void* p, size_t n, void* user) {
  auto* v = static_cast<std::vector<int64_t>*>(user);
  CHECK(n == 16);
  int64_t a[2];
  std::memcpy(a, p, 16);
  CHECK(a[1] == a[0] * 7);
  v->push_back(seq);
  return 0;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/st_selftest";
  // CRC32C known answer + hw == sw
  CHECK(st_crc32c("123456789", 9, 0) == 0xE3069283u);
  std::vector<uint8_t> buf(4099);
  for (size_t i = 0; i < buf.size(); ++i) buf[i] = (uint8_t)(i * 131 + 7);
  CHECK(st_crc32c(buf.data(), buf.size(), 0) == st_crc32c_sw(buf.data(), buf.size(), 0));

  // concurrent appends from 4 threads to one journal (the journal's mutex under TSan)
  void* j = st_journal_open(dir.c_str(), "concurrent", 0);
  CHECK(j != nullptr);
  const int T = 4, N = 500;
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([j, t]() {
      for (int i = 0; i < N; ++i) {
        int64_t a[2] = {t * 100000 + i, (t * 100000 + i) * 7};
        CHECK(st_journal_append(j, a, sizeof(a)) > 0);
      }
    });
  for (auto& x : th) x.join();
  CHECK(st_journal_highest(j) == T * N);
  std::vector<int64_t> seqs;
  CHECK(st_journal_replay(j, 1, -1, count_cb, &seqs) == T * N);
  for (size_t i = 0; i < seqs.size(); ++i) CHECK(seqs[i] == (int64_t)i + 1);
  CHECK(st_journal_delete_to(j, 100) == 0);
  seqs.clear();
  CHECK(st_journal_replay(j, 1, -1, count_cb, &seqs) == T * N - 100);
  st_journal_close(j);
  // reopen: state recovered from the file
  j = st_journal_open(dir.c_str(), "concurrent", 0);
  CHECK(st_journal_highest(j) == T * N);
  st_journal_close(j);

  // snapshots
  const char snap[] = "snapshot-payload";
  CHECK(st_snapshot_save(dir.c_str(), "pid", 42, 1000, snap, sizeof(snap)) == 0);
  int64_t s = 0, ts = 0;
  char path[4096];
  CHECK(st_snapshot_latest(dir.c_str(), "pid", -1, &s, &ts, path, sizeof(path)) == 1);
  CHECK(s == 42 && ts == 1000);
  char back[64];
  CHECK(st_snapshot_read(path, back, sizeof(back)) == (int64_t)sizeof(snap));
  CHECK(std::memcmp(back, snap, sizeof(snap)) == 0);

  // checkpoint writer
  std::vector<float> w(1000);
  for (size_t i = 0; i < w.size(); ++i) w[i] = (float)i * 0.5f;
  int64_t step = 7;
  const char* names[2] = {"w", "step"};
  int dtypes[2] = {0, 5};
  int ndims[2] = {2, 1};
  int64_t shapes[3] = {10, 100, 1};
  const void* datas[2] = {w.data(), &step};
  uint64_t nbytes[2] = {w.size() * 4, 8};
  const std::string meta = "{\"k\":1}";
  const std::string p1 = dir + "/a.stck", p2 = dir + "/b.stck";
  const int64_t n1 = st_ckpt_write(p1.c_str(), 2, names, dtypes, ndims, shapes, datas, nbytes, meta.data(),
                                   meta.size(), 0);
  const int64_t n2 = st_ckpt_write(p2.c_str(), 2, names, dtypes, ndims, shapes, datas, nbytes, meta.data(),
                                   meta.size(), 0);
  CHECK(n1 > 0 && n1 == n2);
  std::printf("selftest ok\n");
  return 0;
}

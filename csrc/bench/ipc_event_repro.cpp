// Minimal reproducer for the interprocess-event refusal seen by the HIP-IPC
// slot rings (rnb_amd/parallel/transport.py IpcRing._wait_ipc_event): does
// hipStreamWaitEvent on an opened IPC event ever return an error, and when?
//
// Two processes (forked before either touches HIP). The parent owns an
// interprocess event (hipEventInterprocess | hipEventDisableTiming), sends
// its handle through a pipe, then runs ROUNDS rounds per pattern:
//   done     record on an idle stream, synchronize, then signal the child
//            (the record has completed long before the child's wait)
//   pending  record behind a ~50 us spin kernel, signal at once
//   burst    record + signal back to back with no kernel and no sync (the
//            slot-reuse rate of a one-video-per-call pipeline)
// The child opens the handle once and, per round, calls hipStreamWaitEvent
// on its own stream, then hipEventQuery, and tallies the return codes; it
// acknowledges each round so the parent never re-records an event the child
// has not waited on yet (the ring protocol guarantees the same: a slot's
// "released" event is recorded again only after the producer rewrote and
// republished the slot, i.e. after the producer's wait on the previous
// record).
//
//   hipcc --offload-arch=gfx950 -O2 csrc/bench/ipc_event_repro.cpp -o ipc_event_repro
//   ./ipc_event_repro [rounds]        (scripts/ipc_event_repro.sh)
//
// Finding (round 4, scripts/ipc_event_matrix.py, profiles/r4_ipc_event_matrix.txt):
// the waits this program sees accepted are exactly the event's first 32
// records ("done": 32 of 2000; "pending"/"burst" run after them: 0). The
// process start method, stream kind, torch context and an IPC event of the
// waiting process's own change nothing. The slot rings record each slot's
// event only a few times per run, which is why they never saw a refusal;
// they now replace every slot event after 30 records
// (parallel/transport.py EVENT_ROTATE) so long runs stay GPU-ordered too.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>

__global__ void spin_kernel(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
}

static void check(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    fprintf(stderr, "%s: %s\n", what, hipGetErrorString(e));
    exit(3);
  }
}

static bool read_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    const ssize_t r = read(fd, c, n);
    if (r <= 0) return false;
    c += r;
    n -= (size_t)r;
  }
  return true;
}

static bool write_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    const ssize_t r = write(fd, c, n);
    if (r <= 0) return false;
    c += r;
    n -= (size_t)r;
  }
  return true;
}

static const char* kPatterns[] = {"done", "pending", "burst"};

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
  int to_child[2], to_parent[2];
  if (pipe(to_child) || pipe(to_parent)) return 2;
  const pid_t pid = fork();
  if (pid < 0) return 2;
  if (pid == 0) {
    // ---- child: consumer side --------------------------------------------
    close(to_child[1]);
    close(to_parent[0]);
    check(hipSetDevice(0), "child hipSetDevice");
    hipIpcEventHandle_t h;
    if (!read_all(to_child[0], &h, sizeof(h))) return 4;
    hipEvent_t ev;
    check(hipIpcOpenEventHandle(&ev, h), "hipIpcOpenEventHandle");
    hipStream_t s;
    check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "child stream");
    for (int p = 0; p < 3; ++p) {
      std::map<int, int> wait_rc, query_rc, refused_query;
      for (int r = 0; r < rounds; ++r) {
        char go;
        if (!read_all(to_child[0], &go, 1)) return 5;
        const hipError_t w = hipStreamWaitEvent(s, ev, 0);
        const hipError_t q = hipEventQuery(ev);
        wait_rc[(int)w]++;
        query_rc[(int)q]++;
        if (w != hipSuccess) {
          refused_query[(int)q]++;
          (void)hipGetLastError();
        }
        check(hipStreamSynchronize(s), "child sync");
        const char ack = 1;
        if (!write_all(to_parent[1], &ack, 1)) return 6;
      }
      printf("pattern %-8s rounds %d  hipStreamWaitEvent rc:", kPatterns[p], rounds);
      for (auto& kv : wait_rc) printf(" %s=%d", hipGetErrorName((hipError_t)kv.first), kv.second);
      printf("  hipEventQuery rc:");
      for (auto& kv : query_rc) printf(" %s=%d", hipGetErrorName((hipError_t)kv.first), kv.second);
      if (!refused_query.empty()) {
        printf("  query when the wait was refused:");
        for (auto& kv : refused_query)
          printf(" %s=%d", hipGetErrorName((hipError_t)kv.first), kv.second);
      }
      printf("\n");
      fflush(stdout);
    }
    check(hipStreamDestroy(s), "child stream destroy");
    return 0;
  }
  // ---- parent: producer side ---------------------------------------------
  close(to_child[0]);
  close(to_parent[1]);
  check(hipSetDevice(0), "parent hipSetDevice");
  hipEvent_t ev;
  check(hipEventCreateWithFlags(&ev, hipEventInterprocess | hipEventDisableTiming),
        "hipEventCreateWithFlags");
  hipIpcEventHandle_t h;
  check(hipIpcGetEventHandle(&h, ev), "hipIpcGetEventHandle");
  if (!write_all(to_child[1], &h, sizeof(h))) return 4;
  hipStream_t s;
  check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "parent stream");
  for (int p = 0; p < 3; ++p) {
    for (int r = 0; r < rounds; ++r) {
      if (p == 1) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, 100000LL);
      check(hipEventRecord(ev, s), "hipEventRecord");
      if (p == 0) check(hipStreamSynchronize(s), "parent sync");
      const char go = 1;
      if (!write_all(to_child[1], &go, 1)) return 5;
      char ack;
      if (!read_all(to_parent[0], &ack, 1)) return 6;
    }
  }
  check(hipStreamSynchronize(s), "parent final sync");
  int status = 0;
  waitpid(pid, &status, 0);
  check(hipStreamDestroy(s), "parent stream destroy");
  check(hipEventDestroy(ev), "parent event destroy");
  return WIFEXITED(status) ? WEXITSTATUS(status) : 7;
}

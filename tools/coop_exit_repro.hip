// Reproducer for the exit-time SIGSEGV seen under rocprofv3 after a cooperative launch (VERDICT
// r05 W6), with no n2v2r code: one trivial kernel launched with hipLaunchCooperativeKernel
// ("coop") or hipLaunchKernelGGL ("plain"), synchronised, memory freed, return from main.
// At exit (the handler is installed by an atexit callback registered after the runtime and the
// profiler tool initialised, so it runs before their teardown) a SIGSEGV prints
// /proc/self/maps, so the PCs of the crash trace can be mapped to libraries offline.
//   hipcc --offload-arch=gfx950 -O2 tools/coop_exit_repro.hip -o tools/coop_exit_repro
//   rocprofv3 --kernel-trace --stats -d out -- ./tools/coop_exit_repro coop
#include <hip/hip_runtime.h>
#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fcntl.h>
#include <ucontext.h>
#include <unistd.h>

__global__ void mark(int* p) {
  if (threadIdx.x == 0) p[blockIdx.x] = (int)blockIdx.x + 1;
}

static void put_hex(const char* label, unsigned long v) {
  char b[64];
  int n = 0;
  while (label[n]) {
    b[n] = label[n];
    ++n;
  }
  for (int s = 60; s >= 0; s -= 4) b[n++] = "0123456789abcdef"[(v >> s) & 15];
  b[n++] = '\n';
  (void)!write(2, b, (size_t)n);
}

static void dump_maps(int sig, siginfo_t* si, void* ctx) {
  const char hdr[] = "\n[coop_exit_repro] fatal signal at exit\n";
  (void)!write(2, hdr, sizeof(hdr) - 1);
  put_hex("fault address 0x", (unsigned long)si->si_addr);
  put_hex("pc 0x", (unsigned long)static_cast<ucontext_t*>(ctx)->uc_mcontext.gregs[REG_RIP]);
  const char mh[] = "/proc/self/maps:\n";
  (void)!write(2, mh, sizeof(mh) - 1);
  const int fd = open("/proc/self/maps", O_RDONLY);
  char buf[4096];
  for (ssize_t r; fd >= 0 && (r = read(fd, buf, sizeof(buf))) > 0;) (void)!write(2, buf, (size_t)r);
  _exit(128 + sig);
}

static void arm_at_exit() {
  struct sigaction sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = dump_maps;
  sa.sa_flags = SA_SIGINFO;
  sigaction(SIGSEGV, &sa, nullptr);
  const char m[] = "[coop_exit_repro] exit handlers running\n";
  (void)!write(2, m, sizeof(m) - 1);
}

int main(int argc, char** argv) {
  const bool coop = argc > 1 && std::strcmp(argv[1], "coop") == 0;
  int* p = nullptr;
  if (hipMalloc(&p, 64 * sizeof(int)) != hipSuccess) return 2;
  hipError_t e;
  if (coop) {
    void* args[] = {&p};
    e = hipLaunchCooperativeKernel((const void*)mark, dim3(64), dim3(256), args, 0, nullptr);
  } else {
    hipLaunchKernelGGL(mark, dim3(64), dim3(256), 0, nullptr, p);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  int h[64];
  if (e == hipSuccess) e = hipMemcpy(h, p, sizeof(h), hipMemcpyDeviceToHost);
  (void)hipFree(p);
  std::atexit(arm_at_exit);  // after the runtime / tool registered theirs: runs before them
  std::printf("%s launch: %s, p[63] = %d\n", coop ? "cooperative" : "plain", hipGetErrorString(e),
              e == hipSuccess ? h[63] : -1);
  return e == hipSuccess ? 0 : 1;
}

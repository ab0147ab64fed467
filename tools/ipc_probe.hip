// Probe: can two processes on this box share device memory through HIP IPC
// handles (same device: the shared-GPU rehearsal; the async parameter
// server's owner inboxes rely on it)?  Forks BEFORE any HIP call; the parent
// allocates (plain hipMalloc and fine-grained), sends the handles over a
// pipe, the child opens them, writes with a kernel and with a D2D copy, and
// the parent checks the bytes.
//   hipcc --offload-arch=gfx950 -O2 tools/ipc_probe.hip -o build/ipc_probe
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__global__ void fill(unsigned* p, unsigned n, unsigned v) {
  unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v + i;
}

static const unsigned N = 1u << 20;

static int child(int rfd, int wfd) {
  hipIpcMemHandle_t h[2];
  if (read(rfd, h, sizeof(h)) != (ssize_t)sizeof(h)) return 2;
  CK(hipSetDevice(0));
  unsigned* src;
  CK(hipMalloc(&src, N * 4));
  hipLaunchKernelGGL(fill, dim3(N / 256), dim3(256), 0, 0, src, N, 7u);
  for (int k = 0; k < 2; ++k) {
    void* p = nullptr;
    CK(hipIpcOpenMemHandle(&p, h[k], hipIpcMemLazyEnablePeerAccess));
    unsigned* q = static_cast<unsigned*>(p);
    hipLaunchKernelGGL(fill, dim3(N / 512), dim3(256), 0, 0, q, N / 2, 1000u * (k + 1));
    CK(hipMemcpyAsync(q + N / 2, src + N / 2, N * 2, hipMemcpyDeviceToDevice, 0));
    CK(hipDeviceSynchronize());
    CK(hipIpcCloseMemHandle(p));
  }
  char ok = 1;
  if (write(wfd, &ok, 1) != 1) return 3;
  std::printf("child: opened, wrote both buffers\n");
  return 0;
}

int main() {
  int a[2], b[2];
  if (pipe(a) || pipe(b)) return 5;
  pid_t pid = fork();
  if (pid == 0) _exit(child(a[0], b[1]));
  CK(hipSetDevice(0));
  unsigned *p0, *p1;
  CK(hipMalloc(&p0, N * 4));
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&p1), N * 4, hipDeviceMallocFinegrained));
  CK(hipMemset(p0, 0, N * 4));
  CK(hipMemset(p1, 0, N * 4));
  CK(hipDeviceSynchronize());
  hipIpcMemHandle_t h[2];
  CK(hipIpcGetMemHandle(&h[0], p0));
  CK(hipIpcGetMemHandle(&h[1], p1));
  if (write(a[1], h, sizeof(h)) != (ssize_t)sizeof(h)) return 6;
  char ok = 0;
  if (read(b[0], &ok, 1) != 1) std::printf("parent: child gave no ack\n");
  int st = 0;
  waitpid(pid, &st, 0);
  std::printf("child exit %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1);
  static unsigned host[N];
  int bad = 0;
  for (int k = 0; k < 2; ++k) {
    unsigned* p = k ? p1 : p0;
    // a fresh kernel-side read (not only hipMemcpy): copy through a kernel-free D2H
    CK(hipMemcpy(host, p, N * 4, hipMemcpyDeviceToHost));
    int e = 0;
    for (unsigned i = 0; i < N; ++i) {
      unsigned want = i < N / 2 ? 1000u * (k + 1) + i : 7u + i;
      if (host[i] != want) ++e;
    }
    std::printf("%s buffer: %d mismatches\n", k ? "fine-grained" : "hipMalloc", e);
    bad += e;
  }
  std::printf(bad == 0 && ok ? "IPC_OK\n" : "IPC_FAIL\n");
  return bad ? 1 : 0;
}

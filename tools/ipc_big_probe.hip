// ipc_big_probe.hip -- does a HIP IPC mapping of one large allocation work (development aid,
// round 6)?  Two processes: the exporter hipMallocs `bytes`, fills them, publishes the IPC handle
// in <dir>/handle.bin and waits for <dir>/done; the importer opens the handle, copies the last
// GiB (or all, if smaller) out of the mapping and checks it.  Every wait is bounded.
//
//   hipcc -O2 --offload-arch=gfx950 tools/ipc_big_probe.hip -o /tmp/ipc_big_probe
//   /tmp/ipc_big_probe 0 2600000000 /tmp/d & /tmp/ipc_big_probe 1 2600000000 /tmp/d
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool wait_file(const std::string &f, double limit_s) {
    const double t0 = now_s();
    while (access(f.c_str(), F_OK) != 0) {
        if (now_s() - t0 > limit_s) return false;
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
    return true;
}

static int exporter(void *p, size_t bytes, const std::string &hf, const std::string &done) {
    hipIpcMemHandle_t h;
    if (hipIpcGetMemHandle(&h, p) != hipSuccess) { fprintf(stderr, "hipIpcGetMemHandle failed\n"); return 1; }
    const std::string tmp = hf + ".tmp";
    FILE *f = fopen(tmp.c_str(), "wb");
    fwrite(&h, sizeof h, 1, f);
    fclose(f);
    rename(tmp.c_str(), hf.c_str());
    const bool ok = wait_file(done, 60.0);
    printf("exporter %zu bytes: importer %s\n", bytes, ok ? "done" : "did not finish within 60 s");
    fflush(stdout);
    return ok ? 0 : 1;
}

static int importer(size_t bytes, const std::string &hf, const std::string &done) {
    if (!wait_file(hf, 60.0)) { fprintf(stderr, "no handle\n"); return 1; }
    hipIpcMemHandle_t h;
    FILE *f = fopen(hf.c_str(), "rb");
    if (fread(&h, sizeof h, 1, f) != 1) { fclose(f); return 1; }
    fclose(f);
    double t0 = now_s();
    void *src = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&src, h, hipIpcMemLazyEnablePeerAccess);
    const double t_open = now_s() - t0;
    if (e != hipSuccess) { fprintf(stderr, "hipIpcOpenMemHandle: %s\n", hipGetErrorString(e)); return 1; }
    const size_t n = bytes < (1ull << 30) ? bytes : (1ull << 30);
    void *dst = nullptr;
    (void)hipMalloc(&dst, n);
    t0 = now_s();
    const hipError_t ce = hipMemcpy(dst, (char *)src + (bytes - n), n, hipMemcpyDeviceToDevice);
    const double t_copy = now_s() - t0;
    unsigned char last = 0;
    (void)hipMemcpy(&last, (char *)dst + n - 1, 1, hipMemcpyDeviceToHost);
    printf("importer %zu bytes: open %.3f s, copy of the last %zu bytes %s in %.3f s (%.1f GB/s), byte %#x\n", bytes,
           t_open, n, hipGetErrorString(ce), t_copy, n / t_copy / 1e9, last);
    fflush(stdout);
    (void)hipIpcCloseMemHandle(src);
    (void)hipFree(dst);
    FILE *d = fopen(done.c_str(), "w");
    fclose(d);
    return last == 0x5A ? 0 : 1;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s role bytes dir [repeats]\n", argv[0]);
        return 2;
    }
    const int role = atoi(argv[1]);
    const size_t bytes = strtoull(argv[2], nullptr, 10);
    const std::string dir = argv[3];
    const int reps = argc > 4 ? atoi(argv[4]) : 1;
    // role 2 / 3 (exporter / importer, a 5th argument "a,b,c" of sizes): a growing buffer, as a
    // rank's send buffer in a solve -- a new allocation of each size exported in turn, the
    // importer keeping every earlier mapping open
    if (role >= 2) {
        std::vector<size_t> sizes;
        for (char *q = argv[5]; *q;) {
            sizes.push_back(strtoull(q, &q, 10));
            if (*q == ',') q++;
        }
        std::vector<void *> maps;
        for (size_t i = 0; i < sizes.size(); i++) {
            const std::string sfx = "." + std::to_string(i);
            const std::string hf = dir + "/handle" + sfx + ".bin", done = dir + "/done" + sfx;
            if (role == 2) {
                void *q = nullptr;
                if (hipMalloc(&q, sizes[i]) != hipSuccess) { fprintf(stderr, "hipMalloc failed\n"); return 1; }
                (void)hipMemset(q, 0x5A, sizes[i]);
                (void)hipDeviceSynchronize();
                if (exporter(q, sizes[i], hf, done)) return 1;
            } else {
                if (!wait_file(hf, 60.0)) { fprintf(stderr, "no handle %zu\n", i); return 1; }
                hipIpcMemHandle_t h;
                FILE *f = fopen(hf.c_str(), "rb");
                if (fread(&h, sizeof h, 1, f) != 1) { fclose(f); return 1; }
                fclose(f);
                printf("importer: opening %zu bytes (%zu mappings open)\n", sizes[i], maps.size());
                fflush(stdout);
                const double t0 = now_s();
                void *src = nullptr;
                if (hipIpcOpenMemHandle(&src, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return 1;
                printf("importer: opened in %.3f s\n", now_s() - t0);
                fflush(stdout);
                maps.push_back(src);
                FILE *d = fopen(done.c_str(), "w");
                fclose(d);
            }
        }
        for (void *m : maps) (void)hipIpcCloseMemHandle(m);
        return 0;
    }
    void *p = nullptr;
    if (role == 0) {
        if (hipMalloc(&p, bytes) != hipSuccess) { fprintf(stderr, "hipMalloc failed\n"); return 1; }
        (void)hipMemset(p, 0x5A, bytes);
        (void)hipDeviceSynchronize();
    }
    for (int i = 0; i < reps; i++) {
        const std::string sfx = reps > 1 ? "." + std::to_string(i) : "";
        const std::string hf = dir + "/handle" + sfx + ".bin", done = dir + "/done" + sfx;
        const int rc = role == 0 ? exporter(p, bytes, hf, done) : importer(bytes, hf, done);
        if (rc) return rc;
    }
    if (p) (void)hipFree(p);
    return 0;
}

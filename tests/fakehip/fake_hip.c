/* fake_hip.c -- a host-memory stand-in for the HIP runtime calls libbhrt's host C makes, so
 * bhrt_api.c can be driven with SEVERAL simulated devices on a machine without a GPU, under
 * ASan/UBSan and TSan (tests/test_multidevice_host.py; VERDICT r1 "multi-device state").
 *
 * Device memory is malloc'ed and tagged with the device that allocated it; every stream
 * operation runs synchronously at enqueue time (a valid schedule of stream order). Checks
 * that catch host-layer bugs: an operation on a stream of another device than the current
 * one, a device pointer of device A used on device B, a D2H copy into host memory that is
 * neither pinned nor a synchronous hipMemcpy, any page-locking of caller memory.
 * Violations abort with a message (the test then fails). Test infrastructure only. */
#define _GNU_SOURCE
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct ihipStream_t {
    int dev;
};
struct ihipEvent_t {
    int dev;
    double t;
    int recorded;
    hipStream_t stream;      /* where it was last recorded */
    unsigned long seq;       /* the operation count then   */
};

/* Every stream operation runs at enqueue time, but libbhrt must not rely on that: a
 * device-to-device copy whose source is another device's memory (an xGMI peer read queued on
 * the root's stream) counts as still reading that source until the host has waited for the
 * copy's stream (hipStreamSynchronize, or hipEventSynchronize of an event recorded after the
 * copy). hipFree of such a source aborts: on real HIP, hipFree drains only the owning device's
 * queues, not the peer's that reads it (bhrt_render_frame_gather). */
static unsigned long g_seq;

static int n_devices(void) {
    const char* e = getenv("FAKEHIP_DEVICES");
    return e ? atoi(e) : 2;
}

static _Thread_local int g_dev;
static _Thread_local hipError_t g_last;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

#define FAIL(...)                                          \
    do {                                                   \
        fprintf(stderr, "fake_hip: " __VA_ARGS__);         \
        fputc('\n', stderr);                               \
        abort();                                           \
    } while (0)

/* ---- allocation table: [base, base + size) -> device (-1 = pinned host, -2 = registered) */
typedef struct {
    uintptr_t base;
    size_t size;
    int dev;
    hipStream_t pend_stream; /* a peer copy on this stream may still read it ... */
    unsigned long pend_seq;  /* ... the copy's operation count (0: no pending read) */
} alloc_t;
static alloc_t g_alloc[4096];
static int g_nalloc;

static void track(void* p, size_t n, int dev) {
    pthread_mutex_lock(&g_mu);
    if (g_nalloc == (int)(sizeof g_alloc / sizeof *g_alloc)) FAIL("allocation table full");
    g_alloc[g_nalloc++] = (alloc_t){(uintptr_t)p, n, dev, NULL, 0};
    pthread_mutex_unlock(&g_mu);
}
static int untrack(void* p, int dev) {
    int found = 0;
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nalloc; i++)
        if (g_alloc[i].base == (uintptr_t)p && g_alloc[i].dev == dev) {
            g_alloc[i] = g_alloc[--g_nalloc];
            found = 1;
            break;
        }
    pthread_mutex_unlock(&g_mu);
    return found;
}
/* the kind of the memory at [p, p + n): device id, -1 pinned, -2 registered, -3 plain host */
static int kind_of(const void* p, size_t n) {
    int k = -3;
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nalloc; i++)
        if ((uintptr_t)p >= g_alloc[i].base && (uintptr_t)p + n <= g_alloc[i].base + g_alloc[i].size) {
            k = g_alloc[i].dev;
            break;
        }
    pthread_mutex_unlock(&g_mu);
    return k;
}
/* a peer read of [p, p + n) queued on stream s */
static void mark_peer_read(const void* p, size_t n, hipStream_t s) {
    pthread_mutex_lock(&g_mu);
    const unsigned long q = ++g_seq;
    for (int i = 0; i < g_nalloc; i++)
        if ((uintptr_t)p >= g_alloc[i].base && (uintptr_t)p + n <= g_alloc[i].base + g_alloc[i].size) {
            g_alloc[i].pend_stream = s;
            g_alloc[i].pend_seq = q;
        }
    pthread_mutex_unlock(&g_mu);
}
/* the host waited for stream s up to operation count `upto` */
static void host_waited(hipStream_t s, unsigned long upto) {
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nalloc; i++)
        if (g_alloc[i].pend_seq && g_alloc[i].pend_stream == s && g_alloc[i].pend_seq <= upto)
            g_alloc[i].pend_seq = 0;
    pthread_mutex_unlock(&g_mu);
}
static int peer_read_pending(const void* p) {
    int hit = 0;
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nalloc; i++)
        if (g_alloc[i].base == (uintptr_t)p && g_alloc[i].pend_seq) hit = 1;
    pthread_mutex_unlock(&g_mu);
    return hit;
}
static int overlaps_registration(uintptr_t a, size_t n) {
    int hit = 0;
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nalloc; i++)
        if (g_alloc[i].dev == -2 && a < g_alloc[i].base + g_alloc[i].size && g_alloc[i].base < a + n)
            hit = 1;
    pthread_mutex_unlock(&g_mu);
    return hit;
}

/* ---- the caller's host arrays (declared by the driver): page locks must stay inside one of
 * them, and none may be freed while a lock on it is live (a freed-and-reused page that the
 * runtime still believes registered is how DMA reaches memory nobody pinned) ---- */
static alloc_t g_host[1024];
static int g_nhost;

void fakehip_declare_host(const void* p, size_t n) {
    pthread_mutex_lock(&g_mu);
    if (g_nhost == (int)(sizeof g_host / sizeof *g_host)) FAIL("host array table full");
    g_host[g_nhost++] = (alloc_t){(uintptr_t)p, n, -4, NULL, 0};
    pthread_mutex_unlock(&g_mu);
}
void fakehip_forget_host(const void* p) {
    pthread_mutex_lock(&g_mu);
    for (int i = 0; i < g_nhost; i++)
        if (g_host[i].base == (uintptr_t)p) {
            const uintptr_t a = g_host[i].base, b = a + g_host[i].size;
            for (int k = 0; k < g_nalloc; k++)
                if (g_alloc[k].dev == -2 && g_alloc[k].base < b && a < g_alloc[k].base + g_alloc[k].size)
                    FAIL("caller array %p freed while page-locked", p);
            g_host[i] = g_host[--g_nhost];
            break;
        }
    pthread_mutex_unlock(&g_mu);
}
static int inside_caller_array(uintptr_t a, size_t n) {
    pthread_mutex_lock(&g_mu);
    int ok = g_nhost == 0; /* (no declarations: not checked) */
    for (int i = 0; i < g_nhost; i++)
        if (a >= g_host[i].base && a + n <= g_host[i].base + g_host[i].size) ok = 1;
    pthread_mutex_unlock(&g_mu);
    return ok;
}

int fakehip_kind_of(const void* p, size_t n) { return kind_of(p, n); }
int fakehip_current_device(void) { return g_dev; }

static hipError_t ret(hipError_t e) {
    if (e != hipSuccess) g_last = e;
    return e;
}

hipError_t hipGetDeviceCount(int* n) {
    *n = n_devices();
    return *n > 0 ? hipSuccess : ret(hipErrorNoDevice);
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= n_devices()) return ret(hipErrorInvalidDevice);
    g_dev = d;
    return hipSuccess;
}
hipError_t hipGetDevice(int* d) {
    *d = g_dev;
    return hipSuccess;
}
hipError_t hipGetLastError(void) {
    hipError_t e = g_last;
    g_last = hipSuccess;
    return e;
}
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "no error" : "fake_hip error"; }

hipError_t hipMalloc(void** p, size_t n) {
    *p = malloc(n ? n : 1);
    if (!*p) return ret(hipErrorOutOfMemory);
    memset(*p, 0xA5, n); /* device memory is not zeroed */
    track(*p, n, g_dev);
    return hipSuccess;
}
hipError_t hipFree(void* p) {
    if (!p) return hipSuccess;
    if (peer_read_pending(p))
        FAIL("hipFree of %p while a peer copy queued on another device's stream may still read it", p);
    if (!untrack(p, g_dev)) FAIL("hipFree of %p: not a device-%d allocation", p, g_dev);
    free(p);
    return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned flags) {
    (void)flags;
    *p = malloc(n ? n : 1);
    if (!*p) return ret(hipErrorOutOfMemory);
    track(*p, n, -1);
    return hipSuccess;
}
hipError_t hipHostFree(void* p) {
    if (p && !untrack(p, -1)) FAIL("hipHostFree of %p: not pinned", p);
    free(p);
    return hipSuccess;
}
/* libbhrt page-locks no caller memory since round 3: any registration
 * is a host-layer bug */
hipError_t hipHostRegister(void* p, size_t n, unsigned flags) {
    (void)flags;
    if (((uintptr_t)p & 4095) || (n & 4095)) FAIL("hipHostRegister of an unaligned range");
    if (!inside_caller_array((uintptr_t)p, n))
        FAIL("hipHostRegister of [%p, +%zu): pages outside the caller's arrays", p, n);
    FAIL("hipHostRegister of [%p, +%zu): libbhrt must not page-lock caller memory", p, n);
    if (overlaps_registration((uintptr_t)p, n)) return ret(hipErrorHostMemoryAlreadyRegistered);
    track(p, n, -2);
    return hipSuccess;
}
hipError_t hipHostUnregister(void* p) {
    if (!untrack(p, -2)) FAIL("hipHostUnregister of %p: not registered", p);
    return hipSuccess;
}

static void check_stream(hipStream_t s) {
    if (s && s->dev != g_dev) FAIL("stream of device %d used while device %d is current", s->dev, g_dev);
}
hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned flags) {
    (void)flags;
    *s = (hipStream_t)calloc(1, sizeof(struct ihipStream_t));
    (*s)->dev = g_dev;
    return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t a, int dev) {
    (void)dev;
    *v = a == hipDeviceAttributeMultiprocessorCount ? 256 : 0;
    return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned flags, int priority) {
    (void)priority;
    return hipStreamCreateWithFlags(s, flags);
}
hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi) {
    *lo = 0;
    *hi = -1;
    return hipSuccess;
}
hipError_t hipExtStreamCreateWithCUMask(hipStream_t* s, uint32_t n, const uint32_t* mask) {
    (void)n;
    (void)mask;
    return hipStreamCreateWithFlags(s, 0);
}
hipError_t hipStreamSynchronize(hipStream_t s) {
    check_stream(s);
    host_waited(s, (unsigned long)-1);
    return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned flags) {
    (void)flags;
    check_stream(s);
    /* a wait on another device's event is valid HIP (bhrt_render_frame_gather: the root's
     * copies wait for every peer's render); it must have been recorded */
    if (e->dev != g_dev && !e->recorded) FAIL("cross-device wait on an event never recorded");
    return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* e) {
    *e = (hipEvent_t)calloc(1, sizeof(struct ihipEvent_t));
    (*e)->dev = g_dev;
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned flags) {
    (void)flags;
    return hipEventCreate(e);
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
    check_stream(s);
    if (e->dev != g_dev) FAIL("event of device %d recorded on device %d", e->dev, g_dev);
    e->recorded = 1;
    pthread_mutex_lock(&g_mu);
    e->stream = s;
    e->seq = ++g_seq;
    pthread_mutex_unlock(&g_mu);
    return hipSuccess;
}

/* peer access: device-to-device copies may read a peer's memory once it is enabled from the
 * current device */
static _Thread_local unsigned char g_peer[64][64];
hipError_t hipDeviceCanAccessPeer(int* can, int dev, int peer) {
    *can = dev != peer && dev < n_devices() && peer < n_devices();
    return hipSuccess;
}
hipError_t hipDeviceEnablePeerAccess(int peer, unsigned flags) {
    (void)flags;
    if (peer == g_dev || peer >= n_devices()) return ret(hipErrorInvalidDevice);
    if (g_peer[g_dev][peer]) return ret(hipErrorPeerAccessAlreadyEnabled);
    g_peer[g_dev][peer] = 1;
    return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
    if (e->recorded) host_waited(e->stream, e->seq);
    return hipSuccess;
}
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
    (void)a;
    (void)b;
    *ms = 0.f;
    return hipSuccess;
}

/* device side of a copy must be current-device memory; host side as the kind allows */
static void check_copy(void* dst, const void* src, size_t n, hipMemcpyKind kind, int async) {
    if (kind == hipMemcpyDeviceToHost || kind == hipMemcpyDeviceToDevice) {
        const int k = kind_of(src, n);
        const int peer_ok = kind == hipMemcpyDeviceToDevice && k >= 0 && g_peer[g_dev][k];
        if (k != g_dev && !peer_ok)
            FAIL("copy source %p (%zu B) is not device-%d memory nor an enabled peer's (kind %d)",
                 src, n, g_dev, k);
    }
    if (kind == hipMemcpyHostToDevice || kind == hipMemcpyDeviceToDevice) {
        const int k = kind_of(dst, n);
        if (k != g_dev) FAIL("copy destination %p (%zu B) is not device-%d memory (kind %d)", dst, n, g_dev, k);
    }
    if (kind == hipMemcpyDeviceToHost && async) {
        const int k = kind_of(dst, n);
        if (k != -1 && k != -2) FAIL("async D2H into unregistered host memory %p (%zu B)", dst, n);
    }
}
hipError_t hipMemcpy(void* dst, const void* src, size_t n, hipMemcpyKind kind) {
    check_copy(dst, src, n, kind, 0);
    memcpy(dst, src, n);
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t s) {
    check_stream(s);
    check_copy(dst, src, n, kind, kind == hipMemcpyDeviceToHost);
    if (kind == hipMemcpyDeviceToDevice && kind_of(src, n) != g_dev) mark_peer_read(src, n, s);
    memcpy(dst, src, n);
    return hipSuccess;
}
hipError_t hipMemcpy2DAsync(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                            size_t height, hipMemcpyKind kind, hipStream_t s) {
    check_stream(s);
    if (width > dpitch || width > spitch) FAIL("2-D copy wider than its pitch");
    for (size_t r = 0; r < height; r++) {
        check_copy((char*)dst + r * dpitch, (const char*)src + r * spitch, width, kind,
                   kind == hipMemcpyDeviceToHost);
        memcpy((char*)dst + r * dpitch, (const char*)src + r * spitch, width);
        if (kind == hipMemcpyDeviceToDevice && kind_of((const char*)src + r * spitch, width) != g_dev)
            mark_peer_read((const char*)src + r * spitch, width, s);
    }
    return hipSuccess;
}
hipError_t hipMemcpyPeerAsync(void* dst, int dst_dev, const void* src, int src_dev, size_t n,
                              hipStream_t s) {
    check_stream(s);
    if (kind_of(dst, n) != dst_dev || kind_of(src, n) != src_dev)
        FAIL("peer copy %p (device %d) <- %p (device %d): wrong devices", dst, dst_dev, src, src_dev);
    if (src_dev != g_dev) mark_peer_read(src, n, s);
    memcpy(dst, src, n);
    return hipSuccess;
}
hipError_t hipMemcpy2D(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width,
                       size_t height, hipMemcpyKind kind) {
    if (width > dpitch || width > spitch) FAIL("2-D copy wider than its pitch");
    for (size_t r = 0; r < height; r++) {
        check_copy((char*)dst + r * dpitch, (const char*)src + r * spitch, width, kind, 0);
        memcpy((char*)dst + r * dpitch, (const char*)src + r * spitch, width);
    }
    return hipSuccess;
}
hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t s) {
    check_stream(s);
    if (kind_of(p, n) != g_dev) FAIL("memset of %p: not device-%d memory", p, g_dev);
    memset(p, v, n);
    return hipSuccess;
}

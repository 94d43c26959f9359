/* Bench-only stand-in for the Java producers of the delta-streaming leg (bench.py).
 *
 * In a deployment the RPC threads that run FollowerInfo.updateMatchIndex (FollowerInfoImpl.java:93-105)
 * each write their 16-byte rh_delta straight into the pinned staging slot that rh_deltas_acquire
 * hands out.  bench.py replays that with a pool of persistent native threads that copy their share
 * of a pre-generated step into the slot -- no Python thread-pool dispatch in the timed loop.
 * bp_push replays the Java module's own producer path instead: every thread owns a share of the
 * step's deltas (the divisions / followers whose appender it is) and hands them to
 * rh_node_push_deltas in buffer-sized calls, concurrently with the other threads
 * (HipLeaderBookkeeper.DeltaBuffer, 4096 deltas).
 *
 * Not product code: libratis_hip never links this, and it touches no GPU API.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BP_EXPORT __attribute__((visibility("default")))
#define BP_MAX_THREADS 64

typedef struct bp_pool bp_pool;
typedef struct {
    bp_pool* p;
    int id;
} bp_arg;

/* Workers sleep on a condition variable between rounds (no spinning: a spin-waiting pool would
 * eat the CPU share the main thread and the HIP runtime need). */
struct bp_pool {
    pthread_t th[BP_MAX_THREADS];
    bp_arg arg[BP_MAX_THREADS];
    int n;                  /* worker threads; the caller of bp_fill takes share n of n + 1 */
    pthread_mutex_t mu;
    pthread_cond_t go, fin;
    uint64_t gen;           /* bumped by bp_fill to start a round */
    int done;               /* workers finished with the current round */
    int quit;
    char* dst;
    const char* src;
    size_t bytes;
    /* bp_push rounds */
    int mode;               /* 0: copy (bp_fill), 1: push (bp_push) */
    int (*push)(void*, const void*, size_t);
    void* node;
    const uint64_t* shares; /* [n + 1] record offsets: producer i pushes [shares[i], shares[i + 1]) */
    size_t chunk;           /* records per push call */
    int rc;                 /* first failing push's return code (0: all succeeded) */
};

/* share `id` of `parts`, cut on 16-byte record boundaries */
static void copy_share(bp_pool* p, int id, int parts) {
    const size_t recs = p->bytes / 16;
    const size_t lo = recs * (size_t)id / (size_t)parts * 16;
    const size_t hi = (id == parts - 1) ? p->bytes : recs * (size_t)(id + 1) / (size_t)parts * 16;
    if (hi > lo) memcpy(p->dst + lo, p->src + lo, hi - lo);
}

/* producer `id` pushes its share in calls of `chunk` records */
static void push_share(bp_pool* p, int id) {
    const uint64_t lo = p->shares[id], hi = p->shares[id + 1];
    for (uint64_t i = lo; i < hi; i += p->chunk) {
        const uint64_t k = hi - i < p->chunk ? hi - i : p->chunk;
        const int rc = p->push(p->node, p->src + i * 16, (size_t)k);
        if (rc != 0) {
            __atomic_compare_exchange_n(&p->rc, &(int){0}, rc, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
            return;
        }
    }
}

static void run_share(bp_pool* p, int id) {
    if (p->mode == 1)
        push_share(p, id);
    else
        copy_share(p, id, p->n + 1);
}

static void* worker(void* a) {
    bp_arg* me = (bp_arg*)a;
    bp_pool* p = me->p;
    uint64_t seen = 0;
    pthread_mutex_lock(&p->mu);
    for (;;) {
        while (p->gen == seen && !p->quit) pthread_cond_wait(&p->go, &p->mu);
        if (p->quit) break;
        seen = p->gen;
        pthread_mutex_unlock(&p->mu);
        run_share(p, me->id);
        pthread_mutex_lock(&p->mu);
        if (++p->done == p->n) pthread_cond_signal(&p->fin);
    }
    pthread_mutex_unlock(&p->mu);
    return NULL;
}

/* `threads` producers in all: threads - 1 pool threads plus the thread that calls bp_fill. */
BP_EXPORT void* bp_create(int threads) {
    if (threads < 1) threads = 1;
    if (threads > BP_MAX_THREADS) threads = BP_MAX_THREADS;
    bp_pool* p = (bp_pool*)calloc(1, sizeof(bp_pool));
    if (!p) return NULL;
    pthread_mutex_init(&p->mu, NULL);
    pthread_cond_init(&p->go, NULL);
    pthread_cond_init(&p->fin, NULL);
    for (int i = 0; i < threads - 1; ++i) {
        p->arg[i].p = p;
        p->arg[i].id = i;
        if (pthread_create(&p->th[i], NULL, worker, &p->arg[i]) != 0) break;
        p->n = i + 1;
    }
    return p;
}

/* Copies bytes from src to dst, every producer (pool threads and the caller) taking one
 * contiguous share; returns when all shares are written. */
static void round_wait(bp_pool* p) {
    pthread_mutex_lock(&p->mu);
    while (p->done < p->n) pthread_cond_wait(&p->fin, &p->mu);
    pthread_mutex_unlock(&p->mu);
}

/* Every producer (pool threads and the caller: n + 1 shares) pushes its share of `src` through
 * push(node, records, count) in calls of `chunk` records, all at the same time; returns when all
 * have finished: 0, or the first failing call's return code. */
BP_EXPORT int bp_push(void* pool, void* push, void* node, const void* src, const uint64_t* shares, size_t chunk) {
    bp_pool* p = (bp_pool*)pool;
    if (!p || !push || !chunk) return -1;
    pthread_mutex_lock(&p->mu);
    p->mode = 1;
    p->push = (int (*)(void*, const void*, size_t))push;
    p->node = node;
    p->src = (const char*)src;
    p->shares = shares;
    p->chunk = chunk;
    p->rc = 0;
    p->done = 0;
    p->gen++;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->mu);
    push_share(p, p->n);
    round_wait(p);
    return p->rc;
}

/* Producers in all: the pool threads + the calling thread. */
BP_EXPORT int bp_threads(void* pool) { return pool ? ((bp_pool*)pool)->n + 1 : 0; }

BP_EXPORT int bp_fill(void* pool, void* dst, const void* src, size_t bytes) {
    bp_pool* p = (bp_pool*)pool;
    if (!p) return -1;
    pthread_mutex_lock(&p->mu);
    p->mode = 0;
    p->dst = (char*)dst;
    p->src = (const char*)src;
    p->bytes = bytes;
    p->done = 0;
    p->gen++;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->mu);
    copy_share(p, p->n, p->n + 1);
    pthread_mutex_lock(&p->mu);
    while (p->done < p->n) pthread_cond_wait(&p->fin, &p->mu);
    pthread_mutex_unlock(&p->mu);
    return 0;
}

BP_EXPORT void bp_destroy(void* pool) {
    bp_pool* p = (bp_pool*)pool;
    if (!p) return;
    pthread_mutex_lock(&p->mu);
    p->quit = 1;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->mu);
    for (int i = 0; i < p->n; ++i) pthread_join(p->th[i], NULL);
    pthread_mutex_destroy(&p->mu);
    pthread_cond_destroy(&p->go);
    pthread_cond_destroy(&p->fin);
    free(p);
}

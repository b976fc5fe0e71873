/*
 * rpkt_oracle_mt.c — multi-threaded driver of the CPU oracle (TEST/BASELINE
 * INFRASTRUCTURE ONLY).  Statically partitions the batch over `nthreads`
 * pthreads, each running oracle_parse_batch on its slice: the "all host cores"
 * CPU-baseline leg of SURVEY.md §8d.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include "../include/rpkt_gpu.h"

void oracle_parse_batch(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                        uint32_t stride, uint32_t frame_len, uint32_t n, uint32_t flags,
                        uint32_t n_buckets, rpkt_rec_t* recs, uint64_t* flow_ev);

typedef struct {
    const uint8_t* frames; uint64_t frames_bytes; const uint32_t* offsets;
    uint32_t stride, frame_len, lo, hi, flags, n_buckets; rpkt_rec_t* recs; uint64_t* ev;
} job_t;

static void* run(void* p) {
    job_t* j = (job_t*)p;
    uint32_t cnt = j->hi - j->lo;
    if (j->offsets) {
        oracle_parse_batch(j->frames, j->frames_bytes, j->offsets + j->lo, 0, 0, cnt, j->flags,
                           j->n_buckets, j->recs + j->lo, j->ev ? j->ev + j->lo : NULL);
    } else {
        uint64_t base = (uint64_t)j->lo * j->stride;
        uint64_t fb = j->frames_bytes > base ? j->frames_bytes - base : 0;
        oracle_parse_batch(j->frames + base, fb, NULL, j->stride, j->frame_len, cnt, j->flags,
                           j->n_buckets, j->recs + j->lo, j->ev ? j->ev + j->lo : NULL);
    }
    return NULL;
}

int oracle_parse_batch_mt(const uint8_t* frames, uint64_t frames_bytes, const uint32_t* offsets,
                          uint32_t stride, uint32_t frame_len, uint32_t n, uint32_t flags,
                          uint32_t n_buckets, rpkt_rec_t* recs, uint64_t* flow_ev,
                          int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    if (!th || !jobs) { free(th); free(jobs); return -1; }
    for (int t = 0; t < nthreads; t++) {
        job_t* j = &jobs[t];
        j->frames = frames; j->frames_bytes = frames_bytes; j->offsets = offsets;
        j->stride = stride; j->frame_len = frame_len; j->flags = flags;
        j->n_buckets = n_buckets; j->recs = recs; j->ev = flow_ev;
        j->lo = (uint32_t)((uint64_t)n * t / nthreads);
        j->hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        pthread_create(&th[t], NULL, run, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

/* The same static partition over mbuf chains (config 7's all-cores leg): thread t
 * parses chains [lo, hi) through chain_first + lo (segment indices stay absolute). */
void oracle_parse_chains(const uint8_t* buf, uint64_t buf_bytes, const uint32_t* segs,
                         uint32_t n_segs, const uint32_t* chain_first, uint32_t n_chains,
                         uint32_t flags, uint32_t n_buckets, rpkt_rec_t* recs, uint64_t* flow_ev);

typedef struct {
    const uint8_t* buf; uint64_t buf_bytes; const uint32_t* segs; const uint32_t* first;
    uint32_t n_segs, lo, hi, flags, n_buckets; rpkt_rec_t* recs; uint64_t* ev;
} chain_job_t;

static void* run_chains(void* p) {
    chain_job_t* j = (chain_job_t*)p;
    oracle_parse_chains(j->buf, j->buf_bytes, j->segs, j->n_segs, j->first + j->lo, j->hi - j->lo,
                        j->flags, j->n_buckets, j->recs + j->lo, j->ev ? j->ev + j->lo : NULL);
    return NULL;
}

int oracle_parse_chains_mt(const uint8_t* buf, uint64_t buf_bytes, const uint32_t* segs,
                           uint32_t n_segs, const uint32_t* chain_first, uint32_t n_chains,
                           uint32_t flags, uint32_t n_buckets, rpkt_rec_t* recs,
                           uint64_t* flow_ev, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    chain_job_t* jobs = (chain_job_t*)calloc((size_t)nthreads, sizeof(chain_job_t));
    if (!th || !jobs) { free(th); free(jobs); return -1; }
    for (int t = 0; t < nthreads; t++) {
        chain_job_t* j = &jobs[t];
        j->buf = buf; j->buf_bytes = buf_bytes; j->segs = segs; j->first = chain_first;
        j->n_segs = n_segs; j->flags = flags; j->n_buckets = n_buckets; j->recs = recs;
        j->ev = flow_ev;
        j->lo = (uint32_t)((uint64_t)n_chains * t / nthreads);
        j->hi = (uint32_t)((uint64_t)n_chains * (t + 1) / nthreads);
        pthread_create(&th[t], NULL, run_chains, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
    return 0;
}

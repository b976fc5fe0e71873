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

/* Config 1's loop on every usable host thread (the all-cores figure beside the 1-thread
 * one): each thread makes `reps` passes of packet_l4 over the same
 * n frames, as criterion's b.iter would run once per core
 * (benches/rpkt/rpkt_parse.rs:108-140); returns the failed frames summed over threads. */
uint64_t oracle_packet_l4_loop(const uint8_t* frames, uint32_t n, uint32_t stride, uint32_t len,
                               uint32_t reps, uint32_t want_src, uint32_t want_dst,
                               uint16_t want_ip_ck, uint16_t want_ident, uint16_t want_sport,
                               uint16_t want_dport, uint16_t want_ulen, uint16_t want_udp_ck);

typedef struct {
    const uint8_t* frames; uint32_t n, stride, len, reps, src, dst;
    uint16_t ip_ck, ident, sport, dport, ulen, udp_ck; uint64_t bad;
} l4_job_t;

static void* run_l4(void* p) {
    l4_job_t* j = (l4_job_t*)p;
    j->bad = oracle_packet_l4_loop(j->frames, j->n, j->stride, j->len, j->reps, j->src, j->dst,
                                   j->ip_ck, j->ident, j->sport, j->dport, j->ulen, j->udp_ck);
    return NULL;
}

uint64_t oracle_packet_l4_loop_mt(const uint8_t* frames, uint32_t n, uint32_t stride, uint32_t len,
                                  uint32_t reps, int nthreads, uint32_t want_src, uint32_t want_dst,
                                  uint16_t want_ip_ck, uint16_t want_ident, uint16_t want_sport,
                                  uint16_t want_dport, uint16_t want_ulen, uint16_t want_udp_ck) {
    if (nthreads < 1) nthreads = 1;
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    l4_job_t* jobs = (l4_job_t*)calloc((size_t)nthreads, sizeof(l4_job_t));
    if (!th || !jobs) { free(th); free(jobs); return ~0ull; }
    for (int t = 0; t < nthreads; t++) {
        l4_job_t j = {frames, n, stride, len, reps, want_src, want_dst, want_ip_ck, want_ident,
                      want_sport, want_dport, want_ulen, want_udp_ck, 0};
        jobs[t] = j;
        pthread_create(&th[t], NULL, run_l4, &jobs[t]);
    }
    uint64_t bad = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        bad += jobs[t].bad;
    }
    free(th);
    free(jobs);
    return bad;
}

/* Test-only instruments (mog-asr_amd/csrc/testlib/instruments.hip, built into
 * mog_air/_lib/libmog_air_test.so; not part of the product library
 * libmog_air.so).  Loaded by mog_air.ops.spin / lds_poison for the
 * stream-ordering and LDS-hygiene tests (tests/test_gpu_streams.py,
 * scripts/stn_concurrency.py). */
#ifndef MOG_AIR_TEST_H
#define MOG_AIR_TEST_H
#ifdef __cplusplus
extern "C" {
#endif

/* One wave occupying `stream` for `ticks` of the 100 MHz wall clock (<= 1 s):
 * the stream-ordering tests hold one stream of a forked step back with it. */
int mog_spin(long long ticks, void* stream);
/* Fills the LDS of every CU with the 32-bit pattern `bits` (a NaN, say), so a
 * kernel launched next that reads LDS it did not write shows it. */
int mog_lds_poison(unsigned bits, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MOG_AIR_TEST_H */

/* Page-cache write bandwidth of one file: pwrite vs memcpy into a shared
   mapping, T threads, 32 MB blocks (round-5 probe for burg_run_npy).
   gcc -O2 -pthread file_write_probe.c; ./a.out PATH THREADS MODE(0 pwrite, 1 mmap) MB */
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>
static size_t B = 32u << 20, N;
static char *src, *map;
static int fd, NT, mode;
static double now() { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }
static void *work(void *a) {
  long k = (long)a;
  for (size_t i = k; i < N; i += NT) {
    if (mode == 0) { if (pwrite(fd, src, B, i * B) != (ssize_t)B) abort(); }
    else memcpy(map + i * B, src, B);
  }
  return 0;
}
int main(int argc, char **argv) {
  const char *path = argv[1]; NT = atoi(argv[2]); mode = atoi(argv[3]);
  size_t total = (size_t)atol(argv[4]) << 20; N = total / B;
  src = malloc(B); memset(src, 1, B);
  double t0 = now();
  fd = open(path, O_CREAT | O_TRUNC | O_RDWR, 0644);
  if (mode) { if (ftruncate(fd, total)) abort(); map = mmap(0, total, PROT_WRITE, MAP_SHARED, fd, 0); if (map == MAP_FAILED) abort(); }
  pthread_t th[64];
  for (long k = 0; k < NT; ++k) pthread_create(&th[k], 0, work, (void *)k);
  for (int k = 0; k < NT; ++k) pthread_join(th[k], 0);
  if (mode) munmap(map, total);
  close(fd);
  double el = now() - t0;
  printf("mode %s threads %d: %.2f GB/s\n", mode ? "mmap" : "pwrite", NT, total / el / 1e9);
  unlink(path);
  return 0;
}

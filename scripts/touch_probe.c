#define _GNU_SOURCE
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>
#include <stdint.h>
static uint8_t *buf; static size_t N; static int T;
static void *work(void *a){ long i=(long)a; size_t per=N/T; memset(buf+i*per,1,per); return 0; }
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec+t.tv_nsec*1e-9;}
int main(int c,char**v){ N=(size_t)atol(v[1])<<20; int thp=atoi(v[3]);
 for(T=1;T<=atoi(v[2]);T*=2){ buf=malloc(N); if(thp) madvise((void*)(((uintptr_t)buf+(2<<20)-1)&~(uintptr_t)((2<<20)-1)), N-(2<<20), MADV_HUGEPAGE);
 pthread_t th[64]; double t0=now(); for(long i=0;i<T;i++) pthread_create(&th[i],0,work,(void*)i); for(int i=0;i<T;i++) pthread_join(th[i],0);
 double t=now()-t0; printf("thp %d threads %2d: %.1f GB/s first touch\n",thp,T,N/t/1e9); free(buf);} }

/* open(absolute path) vs openat(directory fd, name) + one 4 KiB pread + close, per file, on
 * tmpfs: the path walk the readers repeat for every file of a directory.
 * gcc -O2 -o open_probe open_probe.c && ./open_probe <nfiles> <directory> */
#define _GNU_SOURCE
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>
#include <sys/stat.h>
static double now(){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec+t.tv_nsec*1e-9;}
int main(int argc,char**argv){
  int n=atoi(argv[1]); const char* dir=argv[2];
  char p[512]; char buf[8192];
  mkdir(dir,0755);
  for(int i=0;i<n;i++){snprintf(p,sizeof p,"%s/f%07d",dir,i);int fd=open(p,O_CREAT|O_WRONLY|O_TRUNC,0644);write(fd,buf,4096);close(fd);}
  for(int rep=0;rep<3;rep++){
  double t0=now();
  for(int i=0;i<n;i++){snprintf(p,sizeof p,"%s/f%07d",dir,i);int fd=open(p,O_RDONLY|O_CLOEXEC);pread(fd,buf,4096,0);close(fd);}
  double t1=now();
  int d=open(dir,O_PATH|O_DIRECTORY|O_CLOEXEC);
  for(int i=0;i<n;i++){snprintf(p,sizeof p,"f%07d",i);int fd=openat(d,p,O_RDONLY|O_CLOEXEC);pread(fd,buf,4096,0);close(fd);}
  double t2=now(); close(d);
  printf("abs %.3f us/file  openat %.3f us/file\n",(t1-t0)/n*1e6,(t2-t1)/n*1e6);}
  for(int i=0;i<n;i++){snprintf(p,sizeof p,"%s/f%07d",dir,i);unlink(p);} rmdir(dir);
}

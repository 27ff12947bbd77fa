/* fuse_probe.c — can this host serve a kernel FUSE mount?  (VERDICT r1,
 * Missing 5: "if mount(2) of /dev/fuse is refused, record the errno".)
 *
 * Opens /dev/fuse, then tries the raw mount(2) a FUSE daemon performs
 * (filesystem type "fuse", fd=<dev fd>, rootmode, user_id, group_id), and
 * looks for the setuid helper fusermount(3) a non-root daemon would use.
 * Prints one JSON line; never leaves a mount behind (a successful mount is
 * unmounted at once with umount2(MNT_DETACH)).
 *
 * build: gcc -O2 -o tools/fuse_probe tools/fuse_probe.c */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mount.h>
#include <sys/stat.h>
#include <unistd.h>

static const char *which(const char *name) {
  static char buf[512];
  const char *dirs[] = {"/bin", "/usr/bin", "/sbin", "/usr/sbin", "/usr/local/bin", NULL};
  for (int i = 0; dirs[i]; ++i) {
    snprintf(buf, sizeof buf, "%s/%s", dirs[i], name);
    if (access(buf, X_OK) == 0) return buf;
  }
  return NULL;
}

int main(void) {
  char dir[] = "/tmp/bfrs_fuse_probe_XXXXXX";
  int open_errno = 0, mount_errno = 0, mounted = 0;
  const int fd = open("/dev/fuse", O_RDWR | O_CLOEXEC);
  if (fd < 0) open_errno = errno;
  if (!mkdtemp(dir)) {
    printf("{\"error\": \"mkdtemp: %s\"}\n", strerror(errno));
    return 1;
  }
  if (fd >= 0) {
    char opts[128];
    snprintf(opts, sizeof opts, "fd=%d,rootmode=40000,user_id=%u,group_id=%u", fd, getuid(),
             getgid());
    if (mount("bfrs_probe", dir, "fuse", MS_NOSUID | MS_NODEV | MS_RDONLY, opts) == 0) {
      mounted = 1;
      umount2(dir, MNT_DETACH);
    } else {
      mount_errno = errno;
    }
    close(fd);
  }
  rmdir(dir);
  const char *fm = which("fusermount3");
  if (!fm) fm = which("fusermount");
  struct stat st;
  const int have_dev = stat("/dev/fuse", &st) == 0;
  printf("{\"uid\": %u, \"dev_fuse\": %s, \"open_errno\": %d, \"open_error\": \"%s\", "
         "\"mount_errno\": %d, \"mount_error\": \"%s\", \"mounted\": %s, \"fusermount\": %s%s%s}\n",
         getuid(), have_dev ? "true" : "false", open_errno, open_errno ? strerror(open_errno) : "",
         mount_errno, mount_errno ? strerror(mount_errno) : "", mounted ? "true" : "false",
         fm ? "\"" : "", fm ? fm : "null", fm ? "\"" : "");
  return 0;
}

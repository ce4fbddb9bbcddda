// Child processes without Python's subprocess module.
//
// The reference shells out to external tools with os/exec (operator-sdk in
// internal/transformer/k8stransformer.go:226-247, podman/docker in
// internal/containerizer/cnb/containerruntimeprovider.go:45-130, cf/kubectl in
// internal/collector/*.go).  A Go binary pays one fork+exec per tool; a cold
// Python process pays that plus ~2 ms to import subprocess (selectors, signal,
// threading glue) and a GIL-bound fork path.  These two entry points are what
// move2kube_amd/utils/proc.py needs instead:
//
//   proc_spawn(argv, cwd, stdout, stderr) -> (pid, out_rfd, err_rfd)
//       posix_spawnp (glibc: clone(CLONE_VM|CLONE_VFORK), so the parent's
//       address-space size does not matter) with stdin on /dev/null and
//       SIGPIPE/SIGXFSZ reset to default and descriptors above 2 closed in
//       the child, as subprocess does.
//       stdout: -1 pipe, -2 /dev/null, -3 inherit, >= 0 that descriptor.
//       stderr: the same codes, plus -4 = into stdout.
//       Failure raises OSError(errno, strerror, argv[0]) like subprocess.
//   proc_wait(pid, out_rfd, err_rfd, timeout_s) -> (returncode, out, err, timed_out)
//       Drains the pipes and reaps the child with the GIL released; a pidfd
//       wakes the wait when the child exits after closing its pipes.  On
//       timeout (> 0) the child is SIGKILLed and reaped.  returncode follows
//       subprocess (-N for signal N).  A pending Python signal (Ctrl-C) kills
//       the child and is raised.

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cerrno>
#include <csignal>
#include <cstring>
#include <fcntl.h>
#include <poll.h>
#include <spawn.h>
#include <string>
#include <sys/syscall.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>
#include <vector>

extern char **environ;

namespace {

enum : long { FD_PIPE = -1, FD_DEVNULL = -2, FD_INHERIT = -3, FD_STDOUT = -4 };

double mono_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

bool bytes_arg(PyObject *o, std::string &out) {
  if (PyBytes_Check(o)) {
    out.assign(PyBytes_AS_STRING(o), (size_t)PyBytes_GET_SIZE(o));
    return true;
  }
  if (PyUnicode_Check(o)) {
    PyObject *b = PyUnicode_EncodeFSDefault(o);
    if (!b) return false;
    out.assign(PyBytes_AS_STRING(b), (size_t)PyBytes_GET_SIZE(b));
    Py_DECREF(b);
    return true;
  }
  PyErr_SetString(PyExc_TypeError, "expected bytes or str");
  return false;
}

void close_quiet(int &fd) {
  if (fd >= 0) close(fd);
  fd = -1;
}

int pidfd_for(pid_t pid) {
#ifdef SYS_pidfd_open
  long r = syscall(SYS_pidfd_open, pid, 0);
  if (r >= 0) {
    fcntl((int)r, F_SETFD, FD_CLOEXEC);
    return (int)r;
  }
#endif
  return -1;
}

int returncode_of(int status) {
  if (WIFEXITED(status)) return WEXITSTATUS(status);
  if (WIFSIGNALED(status)) return -WTERMSIG(status);
  return 0;
}

}  // namespace

extern "C" PyObject *m2k_proc_spawn(PyObject *argv_obj, PyObject *cwd_obj, long out_mode, long err_mode) {
  if (!PyList_Check(argv_obj) || PyList_GET_SIZE(argv_obj) == 0) {
    PyErr_SetString(PyExc_ValueError, "argv must be a non-empty list");
    return nullptr;
  }
  std::vector<std::string> args((size_t)PyList_GET_SIZE(argv_obj));
  for (Py_ssize_t i = 0; i < PyList_GET_SIZE(argv_obj); i++)
    if (!bytes_arg(PyList_GET_ITEM(argv_obj, i), args[(size_t)i])) return nullptr;
  for (auto &a : args)
    if (a.find('\0') != std::string::npos) {
      PyErr_SetString(PyExc_ValueError, "embedded null byte");
      return nullptr;
    }
  std::string cwd;
  if (cwd_obj != Py_None && !bytes_arg(cwd_obj, cwd)) return nullptr;

  int opipe[2] = {-1, -1}, epipe[2] = {-1, -1};
  auto fail_errno = [&](int e) -> PyObject * {
    close_quiet(opipe[0]);
    close_quiet(opipe[1]);
    close_quiet(epipe[0]);
    close_quiet(epipe[1]);
    errno = e;
    PyObject *name = PyUnicode_DecodeFSDefaultAndSize(args[0].data(), (Py_ssize_t)args[0].size());
    PyErr_SetFromErrnoWithFilenameObject(PyExc_OSError, name);
    Py_XDECREF(name);
    return nullptr;
  };
  if (out_mode == FD_PIPE && pipe2(opipe, O_CLOEXEC) != 0) return fail_errno(errno);
  if (err_mode == FD_PIPE && pipe2(epipe, O_CLOEXEC) != 0) return fail_errno(errno);

  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  if (out_mode == FD_PIPE)
    posix_spawn_file_actions_adddup2(&fa, opipe[1], 1);
  else if (out_mode == FD_DEVNULL)
    posix_spawn_file_actions_addopen(&fa, 1, "/dev/null", O_WRONLY, 0);
  else if (out_mode >= 0)
    posix_spawn_file_actions_adddup2(&fa, (int)out_mode, 1);
  if (err_mode == FD_PIPE)
    posix_spawn_file_actions_adddup2(&fa, epipe[1], 2);
  else if (err_mode == FD_DEVNULL)
    posix_spawn_file_actions_addopen(&fa, 2, "/dev/null", O_WRONLY, 0);
  else if (err_mode == FD_STDOUT)
    posix_spawn_file_actions_adddup2(&fa, 1, 2);
  else if (err_mode >= 0)
    posix_spawn_file_actions_adddup2(&fa, (int)err_mode, 2);
  if (!cwd.empty()) posix_spawn_file_actions_addchdir_np(&fa, cwd.c_str());
#if defined(__GLIBC__) && (__GLIBC__ > 2 || (__GLIBC__ == 2 && __GLIBC_MINOR__ >= 34))
  // like subprocess's close_fds=True: the child keeps only 0, 1 and 2, even of
  // descriptors someone opened without O_CLOEXEC
  posix_spawn_file_actions_addclosefrom_np(&fa, 3);
#endif

  posix_spawnattr_t attr;
  posix_spawnattr_init(&attr);
  sigset_t defs;
  sigemptyset(&defs);
  sigaddset(&defs, SIGPIPE);
  sigaddset(&defs, SIGXFSZ);
  posix_spawnattr_setsigdefault(&attr, &defs);
  posix_spawnattr_setflags(&attr, POSIX_SPAWN_SETSIGDEF);

  std::vector<char *> cargv;
  for (auto &a : args) cargv.push_back(const_cast<char *>(a.c_str()));
  cargv.push_back(nullptr);
  pid_t pid = -1;
  int rc;
  Py_BEGIN_ALLOW_THREADS
  rc = posix_spawnp(&pid, cargv[0], &fa, &attr, cargv.data(), environ);
  Py_END_ALLOW_THREADS
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&attr);
  close_quiet(opipe[1]);
  close_quiet(epipe[1]);
  if (rc != 0) return fail_errno(rc);
  return Py_BuildValue("(iii)", (int)pid, opipe[0], epipe[0]);
}

extern "C" PyObject *m2k_proc_wait(long pid_l, long out_fd_l, long err_fd_l, double timeout_s) {
  pid_t pid = (pid_t)pid_l;
  int fds[2] = {(int)out_fd_l, (int)err_fd_l};
  std::string bufs[2];
  int pidfd = pidfd_for(pid);
  const double deadline = timeout_s > 0 ? mono_s() + timeout_s : 0;
  bool timed_out = false, reaped = false;
  int status = 0;
  int interrupted = 0;
  Py_BEGIN_ALLOW_THREADS
  for (;;) {
    if (!reaped) {
      pid_t w = waitpid(pid, &status, WNOHANG);
      if (w == pid || (w < 0 && errno == ECHILD)) reaped = true;
    }
    if (reaped && fds[0] < 0 && fds[1] < 0) break;
    struct pollfd pf[3];
    int n = 0, idx[3];
    for (int k = 0; k < 2; k++)
      if (fds[k] >= 0) {
        pf[n] = {fds[k], POLLIN, 0};
        idx[n++] = k;
      }
    if (!reaped && pidfd >= 0) {
      pf[n] = {pidfd, POLLIN, 0};
      idx[n++] = 2;
    }
    int wait_ms = (!reaped && pidfd < 0) ? 2 : 100;  // no pidfd: poll the child's exit
    if (reaped && n == 0) break;
    if (deadline > 0) {
      double left = deadline - mono_s();
      if (left <= 0) {
        if (!reaped) {
          kill(pid, SIGKILL);
          waitpid(pid, &status, 0);
          reaped = true;
        }
        timed_out = true;
        break;
      }
      if (left * 1000 < wait_ms) wait_ms = (int)(left * 1000) + 1;
    }
    int pr = poll(pf, (nfds_t)n, wait_ms);
    if (pr < 0 && errno == EINTR) {
      Py_BLOCK_THREADS
      interrupted = PyErr_CheckSignals();
      Py_UNBLOCK_THREADS
      if (interrupted) {
        if (!reaped) {
          kill(pid, SIGKILL);
          waitpid(pid, &status, 0);
        }
        break;
      }
      continue;
    }
    for (int j = 0; j < n && pr > 0; j++) {
      if (idx[j] == 2 || !(pf[j].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      int k = idx[j];
      char buf[65536];
      ssize_t r = read(fds[k], buf, sizeof(buf));
      if (r > 0)
        bufs[k].append(buf, (size_t)r);
      else if (r == 0 || (errno != EINTR && errno != EAGAIN))
        close_quiet(fds[k]);
    }
  }
  Py_END_ALLOW_THREADS
  close_quiet(fds[0]);
  close_quiet(fds[1]);
  if (pidfd >= 0) close(pidfd);
  if (interrupted) return nullptr;
  return Py_BuildValue("(iy#y#O)", returncode_of(status), bufs[0].data(), (Py_ssize_t)bufs[0].size(),
                       bufs[1].data(), (Py_ssize_t)bufs[1].size(), timed_out ? Py_True : Py_False);
}

// ---------------------------------------------------------------------------
// A group of running children waited for together (utils/proc.run_many):
//
//   procgroup_new() -> group
//   procgroup_add(group, key, pid, out_rfd, err_rfd, timeout_s)
//   procgroup_wait_any(group) -> (key, returncode, out, err, timed_out), or
//       None when the group is empty
//
// One poll() covers the pipes and pidfds of every live member, so all of them
// drain at once (none blocks on a full pipe while another is waited for), each
// member's deadline counts from its add, and wait_any returns the first member
// that has exited and closed its pipes -- the caller can start the next child
// at once.  No threads, no GIL held while waiting.  A group dropped with live
// members kills and reaps them.
// ---------------------------------------------------------------------------

namespace {

struct Member {
  long key;
  pid_t pid;
  int fds[2];
  int pidfd;
  double deadline;  // 0: none
  std::string bufs[2];
  bool reaped = false, timed_out = false;
  int status = 0;
};

struct ProcGroup {
  std::vector<Member> members;
  ~ProcGroup() {
    for (auto &m : members) {
      if (!m.reaped) {
        kill(m.pid, SIGKILL);
        int st;
        waitpid(m.pid, &st, 0);
      }
      close_quiet(m.fds[0]);
      close_quiet(m.fds[1]);
      close_quiet(m.pidfd);
    }
  }
};

const char *kGroupName = "m2k.procgroup";

void group_free(PyObject *cap) {
  delete static_cast<ProcGroup *>(PyCapsule_GetPointer(cap, kGroupName));
}

ProcGroup *group_of(PyObject *cap) {
  return static_cast<ProcGroup *>(PyCapsule_GetPointer(cap, kGroupName));
}

void reap_nohang(Member &m) {
  if (m.reaped) return;
  pid_t w = waitpid(m.pid, &m.status, WNOHANG);
  if (w == m.pid || (w < 0 && errno == ECHILD)) {
    m.reaped = true;
    close_quiet(m.pidfd);
  }
}

void kill_member(Member &m) {
  if (!m.reaped) {
    kill(m.pid, SIGKILL);
    waitpid(m.pid, &m.status, 0);
    m.reaped = true;
    close_quiet(m.pidfd);
  }
}

}  // namespace

extern "C" PyObject *m2k_procgroup_new() {
  return PyCapsule_New(new ProcGroup(), kGroupName, group_free);
}

extern "C" PyObject *m2k_procgroup_add(PyObject *cap, long key, long pid, long out_fd, long err_fd,
                                       double timeout_s) {
  ProcGroup *g = group_of(cap);
  if (!g) return nullptr;
  Member m;
  m.key = key;
  m.pid = (pid_t)pid;
  m.fds[0] = (int)out_fd;
  m.fds[1] = (int)err_fd;
  m.pidfd = pidfd_for(m.pid);
  m.deadline = timeout_s > 0 ? mono_s() + timeout_s : 0;
  g->members.push_back(std::move(m));
  Py_RETURN_NONE;
}

extern "C" PyObject *m2k_procgroup_wait_any(PyObject *cap) {
  ProcGroup *g = group_of(cap);
  if (!g) return nullptr;
  if (g->members.empty()) Py_RETURN_NONE;
  size_t done = (size_t)-1;
  int interrupted = 0;
  Py_BEGIN_ALLOW_THREADS
  std::vector<struct pollfd> pf;
  std::vector<std::pair<size_t, int>> who;  // (member, 0/1 pipe, 2 pidfd)
  for (;;) {
    for (size_t i = 0; i < g->members.size() && done == (size_t)-1; i++) {
      Member &m = g->members[i];
      reap_nohang(m);
      if (m.reaped && m.fds[0] < 0 && m.fds[1] < 0) done = i;
    }
    if (done != (size_t)-1) break;
    double now = mono_s();
    int wait_ms = 100;
    for (size_t i = 0; i < g->members.size() && done == (size_t)-1; i++) {
      Member &m = g->members[i];
      if (m.deadline > 0 && m.deadline <= now) {
        kill_member(m);
        m.timed_out = true;
        done = i;
      } else if (m.deadline > 0 && (m.deadline - now) * 1000 < wait_ms) {
        wait_ms = (int)((m.deadline - now) * 1000) + 1;
      }
      if (!m.reaped && m.pidfd < 0 && wait_ms > 2) wait_ms = 2;  // no pidfd: poll the exit
    }
    if (done != (size_t)-1) break;
    pf.clear();
    who.clear();
    for (size_t i = 0; i < g->members.size(); i++) {
      Member &m = g->members[i];
      for (int k = 0; k < 2; k++)
        if (m.fds[k] >= 0) {
          pf.push_back({m.fds[k], POLLIN, 0});
          who.push_back({i, k});
        }
      if (!m.reaped && m.pidfd >= 0) {
        pf.push_back({m.pidfd, POLLIN, 0});
        who.push_back({i, 2});
      }
    }
    int pr = poll(pf.data(), (nfds_t)pf.size(), wait_ms);
    if (pr < 0 && errno == EINTR) {
      Py_BLOCK_THREADS
      interrupted = PyErr_CheckSignals();
      Py_UNBLOCK_THREADS
      if (interrupted) break;
      continue;
    }
    for (size_t j = 0; j < pf.size() && pr > 0; j++) {
      if (who[j].second == 2 || !(pf[j].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      Member &m = g->members[who[j].first];
      int k = who[j].second;
      char buf[65536];
      ssize_t r = read(m.fds[k], buf, sizeof(buf));
      if (r > 0)
        m.bufs[k].append(buf, (size_t)r);
      else if (r == 0 || (errno != EINTR && errno != EAGAIN))
        close_quiet(m.fds[k]);
    }
  }
  Py_END_ALLOW_THREADS
  if (interrupted) {  // Ctrl-C: every member is killed, as proc_wait does for its one child
    for (auto &m : g->members) kill_member(m);
    return nullptr;
  }
  Member m = std::move(g->members[done]);
  g->members.erase(g->members.begin() + (long)done);
  close_quiet(m.fds[0]);
  close_quiet(m.fds[1]);
  close_quiet(m.pidfd);
  return Py_BuildValue("(liy#y#O)", m.key, returncode_of(m.status), m.bufs[0].data(), (Py_ssize_t)m.bufs[0].size(),
                       m.bufs[1].data(), (Py_ssize_t)m.bufs[1].size(), m.timed_out ? Py_True : Py_False);
}

/*
 * ftrun -- launcher for the MI355X fault-tolerant Allreduce, the replacement of
 *          `mpiexec --with-ft ulfm -np N ./main BUF` (reference run/run_mpi.sh:24-26).
 *
 *   ftrun -np N [--devmap d0,d1,...] [--] prog [args...]
 *   FTAR_PROG=prog ftrun -np N [--devmap ...] [--] [args...]
 *
 * With FTAR_PROG the program path is not on the launcher's command line, so the
 * harness's killer (kill_procs.sh: R-state processes whose command line contains
 * "main", run/kill_procs.sh:12) can never pick the launcher: the ranks run `prog args`.
 *
 * FTAR_PIN_CPUS=1 pins rank r to the r-th CPU of the launcher's affinity set (CPU
 * baseline runs of the host-memory build: one process per core).
 *
 * Creates the job's shared-memory control block, starts N rank processes (one per
 * GPU by default: rank r drives device r % ngpus, or devmap[r]), and reaps them.
 * The launcher itself never touches the GPU and sleeps in sigtimedwait (S state) until a
 * rank exits or a signal arrives.  A rank that dies is detected by its peers through the
 * control block; the launcher only reaps, forwards MPI_Abort to every remaining rank
 * (checked whenever it wakes, at least every 50 ms), and cleans up on SIGTERM
 * (run_mpi.sh's `timeout 30`).
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <errno.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include "../csrc/ftar_ctrl.h"

static pid_t g_pids[FTAR_MAX_RANKS];
static int g_n;
static char g_name[128];
static int g_term;

static void kill_all(void)
{
    for (int i = 0; i < g_n; i++)
        if (g_pids[i] > 0) kill(g_pids[i], SIGKILL);
}

static void usage(void)
{
    fprintf(stderr, "usage: ftrun -np N [--devmap d0,d1,...] [--] prog [args...]\n"
                    "       FTAR_PROG=prog ftrun -np N [--devmap d0,d1,...] [--] [args...]\n");
    exit(2);
}

int main(int argc, char **argv)
{
    int np = -1, ai = 1;
    const char *devmap = getenv("FTAR_DEVMAP");
    while (ai < argc) {
        if ((!strcmp(argv[ai], "-np") || !strcmp(argv[ai], "-n")) && ai + 1 < argc) {
            np = atoi(argv[ai + 1]);
            ai += 2;
        } else if (!strcmp(argv[ai], "--devmap") && ai + 1 < argc) {
            devmap = argv[ai + 1];
            ai += 2;
        } else if (!strcmp(argv[ai], "--")) {
            ai++;
            break;
        } else {
            break;
        }
    }
    const char *prog = getenv("FTAR_PROG");
    if (prog && !*prog) prog = NULL;
    if (np < 1 || np > FTAR_MAX_RANKS || (!prog && ai >= argc)) usage();
    /* the ranks' argv: prog (FTAR_PROG or the first argument) + the remaining arguments */
    int rest = prog ? ai : ai + 1;
    char *rargv[argc - rest + 2];
    rargv[argc - rest + 1] = NULL;
    rargv[0] = (char *)(prog ? prog : argv[ai]);
    for (int i = rest; i < argc; i++) rargv[1 + i - rest] = argv[i];
    g_n = np;
    snprintf(g_name, sizeof(g_name), "/ftar-job-%d", (int)getpid());
    ftar_job job;
    if (ftar_ctrl_create(&job, g_name, np) != 0) {
        fprintf(stderr, "ftrun: cannot create control block %s\n", g_name);
        return 1;
    }
    atomic_store(&job.shm->launcher_pid, (int)getpid());

    int dev[FTAR_MAX_RANKS];
    for (int r = 0; r < np; r++) dev[r] = -1;
    if (devmap) {
        const char *s = devmap;
        for (int r = 0; r < np && *s; r++) {
            dev[r] = atoi(s);
            while (*s && *s != ',') s++;
            if (*s == ',') s++;
        }
    }

    /* SIGCHLD / SIGTERM / SIGINT are taken synchronously by sigtimedwait below; the
     * children get the default mask and dispositions back before exec */
    sigset_t wset, oldset;
    sigemptyset(&wset);
    sigaddset(&wset, SIGCHLD);
    sigaddset(&wset, SIGTERM);
    sigaddset(&wset, SIGINT);
    sigprocmask(SIG_BLOCK, &wset, &oldset);

    pid_t parent = getpid();
    for (int r = 0; r < np; r++) {
        pid_t pid = fork();
        if (pid < 0) {
            perror("ftrun: fork");
            kill_all();
            shm_unlink(g_name);
            return 1;
        }
        if (pid == 0) {
            sigprocmask(SIG_SETMASK, &oldset, NULL);
            prctl(PR_SET_PDEATHSIG, SIGKILL);
            if (getppid() != parent) _exit(1);
            unsetenv("FTAR_PROG");
            char buf[32];
            setenv("FTAR_JOB", g_name, 1);
            snprintf(buf, sizeof(buf), "%d", r);
            setenv("FTAR_RANK", buf, 1);
            snprintf(buf, sizeof(buf), "%d", np);
            setenv("FTAR_SIZE", buf, 1);
            setenv("FTAR_LAUNCHER", "1", 1);
            if (dev[r] >= 0) {
                snprintf(buf, sizeof(buf), "%d", dev[r]);
                setenv("FTAR_DEVICE", buf, 1);
            }
            const char *pin = getenv("FTAR_PIN_CPUS");
            if (pin && atoi(pin)) {
                cpu_set_t all, one;
                if (sched_getaffinity(0, sizeof(all), &all) == 0 && CPU_COUNT(&all) > 0) {
                    int want = r % CPU_COUNT(&all), k = 0;
                    for (int c = 0; c < CPU_SETSIZE; c++) {
                        if (!CPU_ISSET(c, &all)) continue;
                        if (k++ == want) {
                            CPU_ZERO(&one);
                            CPU_SET(c, &one);
                            (void)sched_setaffinity(0, sizeof(one), &one);
                            break;
                        }
                    }
                }
            }
            execvp(rargv[0], rargv);
            fprintf(stderr, "ftrun: exec %s: %s\n", rargv[0], strerror(errno));
            _exit(127);
        }
        g_pids[r] = pid;
    }

    int alive = np, exit_code = 0, signalled = 0;
    int abort_forwarded = 0;
    while (alive > 0) {
        int st;
        pid_t p = waitpid(-1, &st, WNOHANG);
        if (p == 0) { /* nothing to reap: sleep until a child exits, a signal, or 50 ms */
            struct timespec tmo = {0, 50 * 1000 * 1000};
            int sig = sigtimedwait(&wset, NULL, &tmo);
            if (sig == SIGTERM || sig == SIGINT) g_term = 1;
            p = waitpid(-1, &st, WNOHANG);
        }
        if (p > 0) {
            int who = -1;
            for (int r = 0; r < np; r++)
                if (g_pids[r] == p) {
                    g_pids[r] = -1;
                    who = r;
                }
            alive--;
            if (WIFSIGNALED(st)) signalled++;
            if (WIFSIGNALED(st) && who >= 0 && !atomic_load(&job.shm->abort_flag)) {
                /* post mortem of a killed rank (kill_procs.sh's SIGKILL, an injected kill):
                 * its control slot says what its stream was running when it died */
                int inf = atomic_load(&job.shm->slot[who].inflight);
                fprintf(stderr, "ftrun: rank %d (pid %d) killed by signal %d %s\n", who, (int)p, WTERMSIG(st),
                        inf == FTAR_INFLIGHT_PULL    ? "mid-exchange: a kernel reading peers' HBM in flight"
                        : inf == FTAR_INFLIGHT_LOCAL ? "with a local kernel in flight"
                                                     : "between kernels (no kernel in flight)");
            }
            else if (WIFEXITED(st) && WEXITSTATUS(st) != 0 && !exit_code) exit_code = WEXITSTATUS(st);
            continue;
        }
        if (g_term) {
            kill_all();
            while (waitpid(-1, NULL, 0) > 0) {
            }
            shm_unlink(g_name);
            return 124;
        }
        if (!abort_forwarded && atomic_load(&job.shm->abort_flag)) {
            /* MPI_Abort kills the whole job */
            struct timespec ts = {0, 20 * 1000 * 1000};
            nanosleep(&ts, NULL);
            kill_all();
            abort_forwarded = 1;
        }
    }
    int aborted = atomic_load(&job.shm->abort_flag);
    int code = aborted ? atomic_load(&job.shm->abort_code) : exit_code;
    shm_unlink(g_name);
    if (!code && signalled == np) code = 128 + SIGKILL; /* every rank died: nobody finished */
    /* otherwise some ranks died and the survivors finished cleanly: tolerated, 0 */
    return code;
}

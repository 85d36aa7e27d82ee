/*
 * ftrun -- launcher for the MI355X fault-tolerant Allreduce, the replacement of
 *          `mpiexec --with-ft ulfm -np N ./main BUF` (reference run/run_mpi.sh:24-26).
 *
 *   ftrun -np N [--devmap d0,d1,...] [--] prog [args...]
 *
 * FTAR_PIN_CPUS=1 pins rank r to the r-th CPU of the launcher's affinity set (CPU
 * baseline runs of the host-memory build: one process per core).
 *
 * Creates the job's shared-memory control block, starts N rank processes (one per
 * GPU by default: rank r drives device r % ngpus, or devmap[r]), and reaps them.
 * The launcher itself never touches the GPU and sleeps in waitpid, so the harness's
 * kill_procs.sh (which only shoots R-state processes whose command line contains
 * "main", run/kill_procs.sh:12) never picks it.  A rank that dies is detected by its
 * peers through the control block; the launcher only reaps, forwards MPI_Abort to
 * every remaining rank, and cleans up on SIGTERM (run_mpi.sh's `timeout 30`).
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
static volatile sig_atomic_t g_term;

static void on_term(int sig)
{
    (void)sig;
    g_term = 1;
}

static void kill_all(void)
{
    for (int i = 0; i < g_n; i++)
        if (g_pids[i] > 0) kill(g_pids[i], SIGKILL);
}

static void usage(void)
{
    fprintf(stderr, "usage: ftrun -np N [--devmap d0,d1,...] [--] prog [args...]\n");
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
    if (np < 1 || np > FTAR_MAX_RANKS || ai >= argc) usage();
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

    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_term;
    sigaction(SIGTERM, &sa, NULL);
    sigaction(SIGINT, &sa, NULL);

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
            prctl(PR_SET_PDEATHSIG, SIGKILL);
            if (getppid() != parent) _exit(1);
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
            execvp(argv[ai], &argv[ai]);
            fprintf(stderr, "ftrun: exec %s: %s\n", argv[ai], strerror(errno));
            _exit(127);
        }
        g_pids[r] = pid;
    }

    int alive = np, exit_code = 0, signalled = 0;
    int abort_forwarded = 0;
    while (alive > 0) {
        int st;
        pid_t p = waitpid(-1, &st, WNOHANG);
        if (p > 0) {
            for (int r = 0; r < np; r++)
                if (g_pids[r] == p) g_pids[r] = -1;
            alive--;
            if (WIFSIGNALED(st)) signalled++;
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
        struct timespec ts = {0, 1000 * 1000};
        nanosleep(&ts, NULL);
    }
    int aborted = atomic_load(&job.shm->abort_flag);
    int code = aborted ? atomic_load(&job.shm->abort_code) : exit_code;
    shm_unlink(g_name);
    if (!code && signalled) code = 0; /* tolerated failures: survivors finished cleanly */
    return code;
}

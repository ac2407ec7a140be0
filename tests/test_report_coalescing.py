"""A tracker reports finished tasks to a long-polling JobTracker in one call
(JobTracker.report); while such a report is in flight, tasks finishing
meanwhile do not make calls of their own: the in-flight reporter sends their
news in its next round (TaskTracker.notify_jobtracker).  Every notification is
delivered, with fewer JobTracker calls than notifications."""
import threading
import time

from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.jobconf import JobConf


def test_reports_in_flight_coalesce_later_news():
    conf = JobConf()
    # long heartbeat long-polls: the tracker stays "polling" through the test
    conf.set_int("hbmr.heartbeat.interval.ms", 2000)
    with LocalCluster(conf, num_trackers=1, cpu_slots=1) as cl:
        tt = cl.trackers[0]
        calls = []
        gate = threading.Event()
        real = tt.jt.report

        def report(status, *a, **kw):
            calls.append(status)
            if len(calls) == 1:
                gate.wait(5)             # the first report is slow
            return real(status, *a, **kw)

        tt.jt.report = report
        # the heartbeat thread is long-polling: news goes by report()
        end = time.time() + 5
        while not tt._polling and time.time() < end:
            time.sleep(0.01)
        assert tt._polling
        first = threading.Thread(target=tt.notify_jobtracker)
        first.start()
        while not calls:
            time.sleep(0.005)
        # three more tasks finish while the first report is in flight
        others = [threading.Thread(target=tt.notify_jobtracker) for _ in range(3)]
        for t in others:
            t.start()
        for t in others:
            t.join(5)
        assert all(not t.is_alive() for t in others)     # they did not wait
        assert len(calls) == 1
        gate.set()
        first.join(5)
        # one more round carried the three: 2 calls for 4 notifications
        assert len(calls) == 2
        assert not tt._reporting and not tt._report_again


class _HookLock:
    """A lock whose release can run a callback once (in the releasing thread)."""

    def __init__(self, inner):
        self.inner = inner
        self.hook = None

    def __enter__(self):
        self.inner.acquire()
        return self

    def __exit__(self, *exc):
        self.inner.release()
        h, self.hook = self.hook, None
        if h is not None:
            h()

    def acquire(self, *a, **kw):
        return self.inner.acquire(*a, **kw)

    def release(self):
        self.inner.release()


def test_news_between_the_reporters_last_check_and_its_exit_is_reported():
    """ADVICE r5 (lost wake-up): a task finishing right after the in-flight
    reporter found no more news, but before it stood down, must not be left
    to the long-poll's timeout — it reports itself at once.  Driven on a bare
    TaskTracker (no threads of its own) with the window forced open: the
    reporter's lock release after its last check runs the late notification."""
    from hbmr.mapred.tasktracker import TaskTracker
    tt = TaskTracker.__new__(TaskTracker)
    lock = _HookLock(threading.Lock())
    tt._lock = lock
    tt._notify_seq = 0
    tt._polling = True
    tt.report_news = True
    tt._reporting = tt._report_again = False
    tt._news = threading.Event()
    tt.name = "tracker_bare"
    rung = []

    class JT:
        def report(self, *a, **kw):
            return {}

        def wakeup(self, name, seq):
            rung.append(seq)

    tt.jt = JT()
    calls = []
    reporter = threading.current_thread()
    late = threading.Thread(target=tt.notify_jobtracker)

    def fire():
        if threading.current_thread() is reporter:
            late.start()
            late.join(5)

    def report_once(seq):
        calls.append(threading.current_thread())
        if len(calls) == 1:
            lock.hook = fire            # the reporter's next release: its last check
        return True

    tt._report_once = report_once
    tt.notify_jobtracker()
    assert not late.is_alive()
    assert calls == [reporter, late]    # the late news was reported, by itself
    assert not tt._reporting and not tt._report_again


def test_a_bulk_launched_batch_of_per_attempt_maps_reports_once():
    """The per-attempt GPU maps of one bulk launch (Pipes GPU executables)
    share a _ReportGroup: successes before the batch's last are queued
    without ringing the JobTracker (their statuses ride on the last one's
    report; the defer timer bounds the wait), a failure rings at once."""
    from hbmr.mapred.tasktracker import TaskTracker, _ReportGroup, _Running

    class _Stub:
        def __init__(self):
            self._news = threading.Event()
            self.armed = 0

        def _arm_defer_flush(self):
            self.armed += 1

    tt = _Stub()
    grp = _ReportGroup(3)
    runs = [_Running(None, None, None) for _ in range(3)]
    for r in runs:
        r.group = grp
    assert TaskTracker._group_wake(tt, runs[0], True) is False
    assert tt._news.is_set() and tt.armed == 1
    assert TaskTracker._group_wake(tt, runs[1], False) is True       # a failure: now
    assert TaskTracker._group_wake(tt, runs[2], True) is True        # the last one
    lone = _Running(None, None, None)
    assert TaskTracker._group_wake(tt, lone, True) is True           # no group

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

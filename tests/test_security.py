"""Security: UGI / doAs, AccessControlList, queue and job ACLs on the
JobTracker (TestJobACLs.java, TestQueueManager.java), job-token shuffle hashes
(TestShuffleJobToken.java) and the authenticated RPC handshake."""
from __future__ import annotations

import pytest

from hbmr import security as SEC
from hbmr.examples.sleepjob import sleep_job_conf
from hbmr.mapred import JobConf
from hbmr.mapred.cluster import LocalCluster
from hbmr.mapred.rpc import JT_METHODS, JobTrackerClient, RpcClient, RpcError, RpcServer


def test_ugi_and_acl():
    u = SEC.UserGroupInformation.create_remote_user("alice", ["eng", "ops"])
    assert SEC.UserGroupInformation.get_current_user().user != "alice"
    with u.do_as():
        assert SEC.UserGroupInformation.get_current_user().user == "alice"
        with SEC.UserGroupInformation.create_remote_user("bob").do_as():
            assert SEC.UserGroupInformation.get_current_user().user == "bob"
        assert SEC.UserGroupInformation.get_current_user().user == "alice"
    assert SEC.AccessControlList("*").is_user_allowed(u)
    assert SEC.AccessControlList("alice,carol").is_user_allowed(u)
    assert not SEC.AccessControlList("carol").is_user_allowed(u)
    assert SEC.AccessControlList(" ops").is_user_allowed(u)
    assert not SEC.AccessControlList("").is_user_allowed(u)
    assert not SEC.AccessControlList("x yz").is_user_allowed(u)


def test_job_token_shuffle_hash():
    tm = SEC.JobTokenSecretManager()
    key = tm.add_job("job_1")
    msg = SEC.shuffle_msg("job_1", "attempt_1_m_000001_0", 3)
    url_hash = SEC.generate_hash(msg, key)
    assert SEC.verify_hash(url_hash, msg, key)
    assert not SEC.verify_hash(url_hash, SEC.shuffle_msg("job_1", "attempt_1_m_000001_0", 4), key)
    reply = SEC.generate_hash(url_hash, key)
    assert SEC.verify_reply(reply, url_hash, key)
    tm.remove_job("job_1")
    with pytest.raises(SEC.AccessControlException):
        tm.key("job_1")


def _acl_conf():
    c = JobConf()
    c.set_boolean("mapred.acls.enabled", True)
    c.set("mapred.queue.names", "default,prod")
    c.set("mapred.queue.prod.acl-submit-job", "alice")
    c.set("mapreduce.cluster.administrators", "root2")
    return c


def test_queue_and_job_acls_in_process():
    conf = _acl_conf()
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        job = sleep_job_conf(maps=1, reduces=0, map_ms=1, base=conf)
        job.set("mapred.job.queue.name", "prod")
        with SEC.UserGroupInformation.create_remote_user("bob").do_as():
            with pytest.raises(SEC.AccessControlException):
                cl.submit_job(job)
        job.set("mapred.job.queue.name", "nosuch")
        with pytest.raises(IOError):
            cl.submit_job(job)
        job.set("mapred.job.queue.name", "prod")
        job.set("mapreduce.job.acl-view-job", "carol")
        long_job = sleep_job_conf(maps=1, reduces=0, map_ms=5000, base=conf)
        long_job.set("mapred.job.queue.name", "prod")
        with SEC.UserGroupInformation.create_remote_user("alice").do_as():
            rj = cl.submit_job(job)
            rj.waitForCompletion()
            assert rj.isSuccessful()
            rj2 = cl.submit_job(long_job)
        jid = str(rj.getID())
        assert cl.jt.jobs[jid].conf.get_user() == "alice"
        for who, ok in (("alice", True), ("carol", True), ("root2", True), ("mallory", False)):
            with SEC.UserGroupInformation.create_remote_user(who).do_as():
                if ok:
                    cl.jt.rpc_job_status(jid)
                else:
                    with pytest.raises(SEC.AccessControlException):
                        cl.jt.rpc_job_status(jid)
        with SEC.UserGroupInformation.create_remote_user("carol").do_as():   # view only
            with pytest.raises(SEC.AccessControlException):
                cl.jt.kill_job(rj2.getID())
        with SEC.UserGroupInformation.create_remote_user("root2").do_as():   # admin
            cl.jt.kill_job(rj2.getID())
        assert rj2.getJobState() == "KILLED"


class _Echo:
    def whoami(self):
        return SEC.UserGroupInformation.get_current_user().user


def test_rpc_user_propagation_and_secret_handshake():
    srv = RpcServer(_Echo(), ["whoami"], host="127.0.0.1", secret=None).start()
    try:
        c = RpcClient(f"127.0.0.1:{srv.port}", secret=None)
        with SEC.UserGroupInformation.create_remote_user("dave").do_as():
            assert c.call("whoami") == "dave"
    finally:
        srv.stop()
    srv = RpcServer(_Echo(), ["whoami"], host="127.0.0.1", secret=b"s3cret").start()
    try:
        good = RpcClient(f"127.0.0.1:{srv.port}", secret=b"s3cret")
        with SEC.UserGroupInformation.create_remote_user("erin").do_as():
            assert good.call("whoami") == "erin"
        with SEC.UserGroupInformation.create_remote_user("frank").do_as():
            assert good.call("whoami") == "frank"   # re-handshakes for the new identity
        with pytest.raises(RpcError):
            RpcClient(f"127.0.0.1:{srv.port}", secret=b"wrong").call("whoami")
        with pytest.raises(RpcError):
            RpcClient(f"127.0.0.1:{srv.port}", secret=None).call("whoami")
    finally:
        srv.stop()


def test_remote_job_client_with_secret_and_acls():
    conf = _acl_conf()
    conf.set("hbmr.rpc.secret", "cluster-key")
    with LocalCluster(conf, num_trackers=1, cpu_slots=2) as cl:
        srv = RpcServer(cl.jt, JT_METHODS, host="127.0.0.1",
                        secret=SEC.rpc_secret(conf)).start()
        try:
            client = JobTrackerClient(f"127.0.0.1:{srv.port}", conf)
            job = sleep_job_conf(maps=1, reduces=0, map_ms=1, base=conf)
            job.set("mapreduce.job.acl-view-job", " ")
            with SEC.UserGroupInformation.create_remote_user("alice").do_as():
                rj = client.submit_job(job)
                rj.waitForCompletion(timeout=60)
                assert rj.isSuccessful()
            jid = str(rj.getID())
            assert cl.jt.jobs[jid].conf.get_user() == "alice"
            with SEC.UserGroupInformation.create_remote_user("mallory").do_as():
                with pytest.raises(RpcError, match="AccessControlException"):
                    client.rpc.call("rpc_job_status", jid)
        finally:
            srv.stop()

"""Security: user identity, access control lists, queue/job ACLs and job tokens.

Behaviour from hadoop-1.0.3/src/core/org/apache/hadoop/security/
(UserGroupInformation.java — login user, ``HADOOP_USER_NAME``, createRemoteUser,
doAs; authorize/AccessControlList.java — ``"user1,user2 group1,group2"``, ``*``
for everyone, a leading space for groups only),
src/mapred/org/apache/hadoop/mapred/{JobACLsManager,QueueManager,ACLsManager}.java
(``mapred.acls.enabled``; ``mapreduce.job.acl-view-job`` /
``mapreduce.job.acl-modify-job``; the job owner and
``mapreduce.cluster.administrators`` always pass; queues from
``mapred.queue.names`` with ``mapred.queue.<q>.acl-submit-job`` /
``acl-administer-jobs``), and security/token + mapreduce/security
(JobTokenSecretManager + SecureShuffleUtils: HMAC of the fetch URL with the
job's secret, echoed back by the server).

Kerberos is out of scope (one node); identities are "simple"
auth: the caller states a user name, and RPC servers configured with a
cluster secret (``hbmr.rpc.secret`` / ``hbmr.rpc.secret.file``) only accept
connections that answer an HMAC challenge with it (the DIGEST token analogue,
see hbmr.mapred.rpc).
"""
from __future__ import annotations

import base64
import contextlib
import functools
import getpass
import grp
import hashlib
import hmac
import os
import pwd
import secrets
import threading

_tl = threading.local()


class AccessControlException(PermissionError):
    pass


class UserGroupInformation:
    def __init__(self, user: str, groups=None):
        self.user = user
        self._groups = list(groups) if groups is not None else None

    def get_user_name(self):
        return self.user

    getUserName = get_user_name  # noqa: N815
    getShortUserName = get_user_name  # noqa: N815

    def get_group_names(self):
        if self._groups is None:
            self._groups = unix_groups(self.user)
        return list(self._groups)

    getGroupNames = get_group_names  # noqa: N815

    @staticmethod
    def get_login_user():
        return UserGroupInformation(os.environ.get("HADOOP_USER_NAME") or _login_name())

    getLoginUser = get_login_user  # noqa: N815

    @staticmethod
    def get_current_user():
        stack = getattr(_tl, "stack", None)
        if stack:
            return stack[-1]
        return UserGroupInformation.get_login_user()

    getCurrentUser = get_current_user  # noqa: N815

    @staticmethod
    def create_remote_user(user, groups=None):
        return UserGroupInformation(user, groups)

    createRemoteUser = create_remote_user  # noqa: N815
    createUserForTesting = create_remote_user  # noqa: N815

    @contextlib.contextmanager
    def do_as(self):
        """``with ugi.do_as(): ...`` runs the block as this user (doAs)."""
        stack = getattr(_tl, "stack", None)
        if stack is None:
            stack = _tl.stack = []
        stack.append(self)
        try:
            yield self
        finally:
            stack.pop()

    def __eq__(self, other):
        return isinstance(other, UserGroupInformation) and other.user == self.user

    def __hash__(self):
        return hash(self.user)

    def __repr__(self):
        return f"UGI({self.user})"


@functools.lru_cache(maxsize=1)
def _login_name():
    try:
        return getpass.getuser()
    except Exception:  # noqa: BLE001
        return str(os.getuid())


def unix_groups(user):
    """ShellBasedUnixGroupsMapping: primary + supplementary groups."""
    try:
        pw = pwd.getpwnam(user)
        return [grp.getgrgid(g).gr_name for g in os.getgrouplist(user, pw.pw_gid)]
    except (KeyError, OSError):
        return []


class AccessControlList:
    """``"u1,u2 g1,g2"``; ``"*"`` = everyone; ``" g1"`` = groups only; ``""`` = nobody."""

    def __init__(self, spec: str = "*"):
        spec = spec if spec is not None else "*"
        self.all = spec.strip() == "*"
        users, _, groups = spec.partition(" ")
        self.users = {u.strip() for u in users.split(",") if u.strip()}
        self.groups = {g.strip() for g in groups.split(",") if g.strip()}

    def is_user_allowed(self, ugi: UserGroupInformation) -> bool:
        if self.all or ugi.user in self.users:
            return True
        return bool(self.groups) and bool(self.groups & set(ugi.get_group_names()))

    isUserAllowed = is_user_allowed  # noqa: N815

    def __str__(self):
        if self.all:
            return "*"
        return ",".join(sorted(self.users)) + " " + ",".join(sorted(self.groups))


# ---------------------------------------------------------------- job / queue ACLs
VIEW_JOB, MODIFY_JOB = "mapreduce.job.acl-view-job", "mapreduce.job.acl-modify-job"
SUBMIT_JOB, ADMINISTER_JOBS = "acl-submit-job", "acl-administer-jobs"


def acls_enabled(conf) -> bool:
    return conf is not None and conf.get_boolean("mapred.acls.enabled", False)


def cluster_admins(conf) -> AccessControlList:
    return AccessControlList(conf.get("mapreduce.cluster.administrators", "") if conf else "")


class QueueManager:
    """Queues and their submit/administer ACLs (QueueManager.java)."""

    def __init__(self, conf):
        self.conf = conf
        names = conf.get("mapred.queue.names", "default") if conf is not None else "default"
        self.queues = [q.strip() for q in names.split(",") if q.strip()]

    def acl(self, queue, op):
        return AccessControlList(self.conf.get(f"mapred.queue.{queue}.{op}", "*"))

    def check_submit(self, queue, ugi):
        if queue not in self.queues:
            raise IOError(f"Queue \"{queue}\" does not exist")
        if acls_enabled(self.conf) and not (self.acl(queue, SUBMIT_JOB).is_user_allowed(ugi) or
                                            cluster_admins(self.conf).is_user_allowed(ugi)):
            raise AccessControlException(
                f"User {ugi.user} cannot perform operation SUBMIT_JOB on queue {queue}.")


def check_job_access(cluster_conf, job_conf, ugi, op):
    """JobACLsManager.checkAccess: owner, cluster admins, queue admins, then the job ACL."""
    if not acls_enabled(cluster_conf):
        return True
    owner = job_conf.get("user.name") or job_conf.get("mapreduce.job.user.name")
    if ugi.user == owner or cluster_admins(cluster_conf).is_user_allowed(ugi):
        return True
    if op == MODIFY_JOB:
        q = job_conf.get("mapred.job.queue.name", "default")
        if QueueManager(cluster_conf).acl(q, ADMINISTER_JOBS).is_user_allowed(ugi) and \
                cluster_conf.get(f"mapred.queue.{q}.{ADMINISTER_JOBS}") is not None:
            return True
    if AccessControlList(job_conf.get(op, "")).is_user_allowed(ugi):
        return True
    verb = "VIEW_JOB" if op == VIEW_JOB else "MODIFY_JOB"
    raise AccessControlException(f"User {ugi.user} cannot perform operation {verb} on "
                                 f"{job_conf.get('mapred.job.id', 'job')}")


# ---------------------------------------------------------------- job tokens
class JobTokenSecretManager:
    """Per-job shuffle secrets (JobTokenSecretManager.java)."""

    def __init__(self):
        self._keys: dict[str, bytes] = {}
        self._lock = threading.Lock()

    def add_job(self, job_id, key: bytes | None = None) -> bytes:
        with self._lock:
            k = self._keys.get(str(job_id))
            if k is None:
                k = self._keys[str(job_id)] = key or secrets.token_bytes(20)
            return k

    def remove_job(self, job_id):
        with self._lock:
            self._keys.pop(str(job_id), None)

    def key(self, job_id) -> bytes:
        with self._lock:
            k = self._keys.get(str(job_id))
        if k is None:
            raise AccessControlException(f"no job token for {job_id}")
        return k


def _b64_hmac(key: bytes, msg: str) -> str:
    return base64.b64encode(hmac.new(key, msg.encode(), hashlib.sha1).digest()).decode()


def shuffle_msg(job_id, map_id, reduce) -> str:
    """The string the reference hashes: the mapOutput URL query."""
    return f"/mapOutput?job={job_id}&map={map_id}&reduce={reduce}"


def generate_hash(msg: str, key: bytes) -> str:
    """SecureShuffleUtils.generateHash (UrlHash header / reply hash)."""
    return _b64_hmac(key, msg)


def verify_hash(h: str, msg: str, key: bytes) -> bool:
    return hmac.compare_digest(h.encode(), generate_hash(msg, key).encode())


def verify_reply(reply_hash: str, url_hash: str, key: bytes) -> bool:
    """The reducer checks the server's reply = HMAC(its own UrlHash)."""
    return verify_hash(reply_hash, url_hash, key)


# ---------------------------------------------------------------- RPC secret
def rpc_secret(conf=None) -> bytes | None:
    """Cluster RPC secret from ``hbmr.rpc.secret``, ``hbmr.rpc.secret.file`` or
    the ``HBMR_RPC_SECRET`` environment variable (None = simple, unauthenticated)."""
    v = conf.get("hbmr.rpc.secret") if conf is not None else None
    f = conf.get("hbmr.rpc.secret.file") if conf is not None else None
    if not v and f and os.path.exists(f):
        with open(f, "rb") as fh:
            return fh.read().strip() or None
    v = v or os.environ.get("HBMR_RPC_SECRET")
    return v.encode() if v else None


def rpc_response(secret: bytes, challenge: bytes, user: str) -> str:
    return hmac.new(secret, challenge + b"\0" + user.encode(), hashlib.sha256).hexdigest()

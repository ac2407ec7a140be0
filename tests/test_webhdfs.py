"""WebHDFS REST API + webhdfs:// FileSystem over a MiniDFSCluster.

Mirrors hadoop-1.0.3/src/test/org/apache/hadoop/hdfs/web/
TestWebHdfsFileSystemContract.java (mkdirs/listing/seek/root dir/response
codes), TestJsonUtil.java (FileStatus JSON) and TestOffsetUrlInputStream.java
(offset reads), plus raw-HTTP checks of the two-step redirect protocol and a
MapReduce job reading and writing webhdfs:// paths."""
import collections
import http.client
import json
import os
import urllib.parse

import pytest

from hbmr import fs as F
from hbmr.dfs.cluster import MiniDFSCluster
from hbmr.dfs.webhdfs import PREFIX, WebHdfsFileSystem, WebHdfsServer
from hbmr.mapred import JobClient
from hbmr.mapred.jobconf import JobConf
from hbmr.models import wordcount


@pytest.fixture
def web(tmp_path):
    conf = JobConf()
    conf.set_int("dfs.block.size", 4096)
    conf.set_int("dfs.replication", 2)
    conf.set("hadoop.proxyuser.alice.users", "bob")
    with MiniDFSCluster(conf, num_datanodes=3, base_dir=str(tmp_path / "dfs")) as cl:
        with WebHdfsServer(cl.name, conf) as srv:
            yield cl, srv, WebHdfsFileSystem(srv.address, conf, user="alice")


def _http(srv, method, path, body=None, **q):
    host, port = srv.address.split(":")
    c = http.client.HTTPConnection(host, int(port), timeout=30)
    url = f"{PREFIX}{urllib.parse.quote(path)}?{urllib.parse.urlencode(q)}"
    c.request(method, url, body=body)
    r = c.getresponse()
    out = r.status, dict(r.getheaders()), r.read()
    c.close()
    return out


def test_namespace_ops_and_status_json(web):
    cl, srv, w = web
    assert w.mkdirs("/test/a/b")
    assert w.exists("/test/a") and w.is_dir("/test/a/b")
    with w.create("/test/a/f.txt") as f:
        f.write(b"hello webhdfs\n" * 1000)
    st = w.get_file_status("/test/a/f.txt")
    assert st.length == 14000 and not st.is_dir and st.block_size == 4096
    assert st.owner == "alice" and st.permission == 0o644 and st.replication == 2
    d = w.get_file_status("/test/a/b")
    assert d.is_dir and d.permission == 0o755 and d.owner == "alice"
    assert w.get_file_status("/").permission == 0o777
    # the same file through hdfs:// (the DFS really holds it)
    with cl.filesystem().open(f"{cl.uri}/test/a/f.txt") as f:
        assert f.read() == b"hello webhdfs\n" * 1000
    names = sorted(os.path.basename(s.path) for s in w.list_status("/test/a"))
    assert names == ["b", "f.txt"]
    # JsonUtil field names on the wire
    code, hdr, body = _http(srv, "GET", "/test/a/f.txt", op="GETFILESTATUS", **{"user.name": "x"})
    j = json.loads(body)["FileStatus"]
    assert code == 200 and hdr["Content-Type"] == "application/json"
    assert set(j) == {"pathSuffix", "type", "length", "owner", "group", "permission",
                      "accessTime", "modificationTime", "blockSize", "replication"}
    assert j["type"] == "FILE" and j["permission"] == "644" and j["pathSuffix"] == ""
    cs = w.get_content_summary("/test")
    assert cs["fileCount"] == 1 and cs["directoryCount"] == 3 and cs["length"] == 14000
    assert w.rename("/test/a/f.txt", "/test/g.txt")
    assert not w.exists("/test/a/f.txt") and w.get_file_status("/test/g.txt").length == 14000
    assert not w.rename("/test/missing", "/test/x")
    assert [s.path.rsplit("/", 1)[1] for s in w.glob_status("/test/*.txt")] == ["g.txt"]
    assert w.get_home_directory() == "/user/alice"
    with pytest.raises(IOError):
        w.delete("/test", recursive=False)          # non-empty
    assert w.delete("/test", recursive=True) and not w.exists("/test")
    assert not w.delete("/", recursive=True)         # the root is never deleted
    assert not w.delete("/nothing")


def test_open_seek_offset_reads_and_redirects(web):
    cl, srv, w = web
    data = bytes(range(256)) * 97                   # 24832 B = 7 blocks of 4 KiB
    with w.create("/d/blob") as f:
        f.write(data)
    with w.open("/d/blob", buffering=8192) as f:
        assert f.read() == data
        for off, ln in ((0, 1), (4095, 2), (4096, 4096), (10000, 7000), (24831, 10)):
            f.seek(off)
            assert f.read(ln) == data[off:off + ln]
    # raw protocol: the NameNode redirects OPEN to a DataNode holding the block
    code, hdr, _ = _http(srv, "GET", "/d/blob", op="OPEN", offset=8192, length=100,
                         **{"user.name": "alice"})
    assert code == 307
    loc = urllib.parse.urlsplit(hdr["Location"])
    assert loc.port != int(srv.address.split(":")[1])
    q = urllib.parse.parse_qs(loc.query)
    assert q["op"] == ["OPEN"] and q["offset"] == ["8192"]
    block_hosts = w.get_file_block_locations("/d/blob", 8192, 1)[0][2]
    dn_port = {h: s.server_address[1] for h, s in srv.dn_httpd.items()}
    assert loc.port in [dn_port[h] for h in block_hosts]
    c = http.client.HTTPConnection(loc.hostname, loc.port)
    c.request("GET", f"{loc.path}?{loc.query}")
    r = c.getresponse()
    assert r.status == 200 and r.read() == data[8192:8292]
    # CREATE: 307 without data at the NameNode, 201 + Location from the DataNode
    code, hdr, _ = _http(srv, "PUT", "/d/new", op="CREATE", **{"user.name": "alice"})
    assert code == 307
    loc = urllib.parse.urlsplit(hdr["Location"])
    c = http.client.HTTPConnection(loc.hostname, loc.port)
    c.request("PUT", f"{loc.path}?{loc.query}", body=b"x" * 5000)
    r = c.getresponse()
    r.read()
    assert r.status == 201 and r.getheader("Location").endswith("/d/new")
    # the first replica of each block lands on the DataNode that took the write
    dn_host = [h for h, p in dn_port.items() if p == loc.port][0]
    for _, _, hosts in w.get_file_block_locations("/d/new", 0, 5000):
        assert hosts[0] == dn_host or dn_host in hosts
    assert w.open("/d/new").read() == b"x" * 5000
    # create without overwrite on an existing file fails
    with pytest.raises(FileExistsError):
        with w.create("/d/new", overwrite=False) as f:
            f.write(b"y")


def test_append_checksum_times_owner_permission_replication(web):
    cl, srv, w = web
    with w.create("/e/f", permission=0o600) as f:
        f.write(b"a" * 5000)
    with w.append("/e/f") as f:
        f.write(b"b" * 3000)
    assert w.open("/e/f").read() == b"a" * 5000 + b"b" * 3000
    st = w.get_file_status("/e/f")
    assert st.permission == 0o600 and st.owner == "alice"
    # MD5-of-MD5-of-CRC32: same bytes, same checksum; hdfs:// agrees
    with w.create("/e/g") as f:
        f.write(b"a" * 5000 + b"b" * 3000)
    alg, raw = w.get_file_checksum("/e/f")
    assert alg == "MD5-of-8MD5-of-512CRC32" and len(raw) == 28
    assert w.get_file_checksum("/e/g") == (alg, raw)
    assert cl.filesystem().get_file_checksum(f"{cl.uri}/e/f") == (alg, raw)
    with w.create("/e/h") as f:
        f.write(b"a" * 8000)
    assert w.get_file_checksum("/e/h")[1] != raw
    w.set_times("/e/f", mtime=1_234_567_000, atime=1_234_000_000)
    st = w.get_file_status("/e/f")
    assert st.modification_time == 1_234_567.0 and st.access_time == 1_234_000.0
    w.set_owner("/e/f", owner="carol", group="staff")
    st = w.get_file_status("/e/f")
    assert (st.owner, st.group) == ("carol", "staff")
    w.set_permission("/e/f", 0o640)
    assert w.get_file_status("/e/f").permission == 0o640
    assert w.set_replication("/e/f", 3) and w.get_file_status("/e/f").replication == 3
    assert not w.set_replication("/e", 1)           # directories have no replication
    # attributes survive a NameNode restart (edit-log replay)
    cl.restart_namenode()
    srv.nn = cl.nn
    st = WebHdfsFileSystem(srv.address, user="alice").get_file_status("/e/f")
    assert (st.owner, st.group, st.permission, st.replication) == ("carol", "staff", 0o640, 3)


def test_response_codes_like_the_reference(web):
    """TestWebHdfsFileSystemContract.testResponseCode."""
    cl, srv, w = web
    assert w.mkdirs("/test/testUrl")
    code, _, body = _http(srv, "GET", "/", op="GETHOMEDIRECTORY", **{"user.name": "alice"})
    assert code == 200 and json.loads(body) == {"Path": "/user/alice"}
    # doAs a user alice may not impersonate → 401; one she may → 200
    code, _, body = _http(srv, "GET", "/", op="GETHOMEDIRECTORY", doas="mallory",
                          **{"user.name": "alice"})
    assert code == 401 and json.loads(body)["RemoteException"]["exception"] == "SecurityException"
    code, _, body = _http(srv, "GET", "/", op="GETHOMEDIRECTORY", doas="bob",
                          **{"user.name": "alice"})
    assert code == 200 and json.loads(body)["Path"] == "/user/bob"
    # setOwner with empty parameters → 400
    code, _, _ = _http(srv, "PUT", "/test/testUrl", op="SETOWNER", **{"user.name": "alice"})
    assert code == 400
    # setReplication on a directory → 200 {"boolean": false}
    code, _, body = _http(srv, "PUT", "/test/testUrl", op="SETREPLICATION",
                          **{"user.name": "alice"})
    assert code == 200 and json.loads(body) == {"boolean": False}
    # status of a missing file → 404 FileNotFoundException
    code, _, body = _http(srv, "GET", "/test/testUrl/non-exist", op="GETFILESTATUS",
                          **{"user.name": "alice"})
    r = json.loads(body)["RemoteException"]
    assert code == 404 and r["javaClassName"] == "java.io.FileNotFoundException"
    with pytest.raises(FileNotFoundError):
        w.get_file_status("/test/testUrl/non-exist")
    with pytest.raises(FileNotFoundError):
        w.open("/no/such/file")
    # setPermission with empty parameters → 200, empty octet-stream, 755
    w.set_permission("/test/testUrl", 0o700)
    code, hdr, body = _http(srv, "PUT", "/test/testUrl", op="SETPERMISSION",
                            **{"user.name": "alice"})
    assert code == 200 and body == b"" and hdr["Content-Type"] == "application/octet-stream"
    assert w.get_file_status("/test/testUrl").permission == 0o755
    # bad op / op on the wrong HTTP method / bad parameter value → 400
    assert _http(srv, "GET", "/", op="NOPE")[0] == 400
    assert _http(srv, "GET", "/", op="MKDIRS")[0] == 400
    assert _http(srv, "GET", "/test", op="GET_BLOCK_LOCATIONS", offset="x")[0] in (400, 404)
    assert _http(srv, "DELETE", "/test", op="DELETE", recursive="maybe")[0] == 400
    # op names and parameter names are case-insensitive
    code, _, body = _http(srv, "GET", "/test", OP="getfilestatus")
    assert code == 200 and json.loads(body)["FileStatus"]["type"] == "DIRECTORY"


def test_delegation_tokens(web):
    cl, srv, w = web
    tok = w.get_delegation_token(renewer="alice")
    wt = WebHdfsFileSystem(srv.address, token=tok)
    assert wt.mkdirs("/tok/dir")
    assert wt.get_file_status("/tok/dir").owner == "alice"   # acts as the token's owner
    assert w.renew_delegation_token(tok) > 0
    with pytest.raises(IOError):
        WebHdfsFileSystem(srv.address, user="eve").renew_delegation_token(tok)
    forged = tok[:-3] + ("AAA" if not tok.endswith("AAA") else "BBB")
    with pytest.raises(PermissionError):
        WebHdfsFileSystem(srv.address, token=forged).get_file_status("/tok")
    w.cancel_delegation_token(tok)
    with pytest.raises(PermissionError):
        wt.get_file_status("/tok")


def test_wordcount_job_reads_and_writes_webhdfs(web, tmp_path):
    cl, srv, w = web
    text = "".join(f"alpha beta w{i % 37} gamma w{i % 5}\n" for i in range(3000))
    with w.create("/in/a.txt") as f:
        f.write(text.encode())
    base = f"webhdfs://{srv.address}"
    assert F.is_dfs(f"{base}/in") and isinstance(F.get_fs(f"{base}/in"), WebHdfsFileSystem)
    job = wordcount.make_job(f"{base}/in", f"{base}/out", reduces=2)
    rj = JobClient.runJob(job, verbose=False)
    assert rj.isSuccessful()
    got = collections.Counter()
    for st in w.list_status("/out"):
        for ln in w.open(st.path).read().decode().splitlines():
            k, v = ln.split("\t")
            got[k] += int(v)
    assert got == collections.Counter(text.split())
    assert w.exists("/out/_SUCCESS") and not w.exists("/out/_temporary")

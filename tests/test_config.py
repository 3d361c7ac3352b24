import os

import pytest

from akka_allreduce_1_amd import config as mc

REF_CONF = "/root/reference/src/main/resources/application.conf"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_hocon_subset():
    t = mc.parse_hocon('''
    # comment
    a { b = 1, c : "x y" // trailing
        d.e = [1, 2, "three"] }
    a.f = true
    g = 10s
    ''')
    flat = mc.flatten(t)
    assert flat == {"a.b": 1, "a.c": "x y", "a.d.e": [1, 2, "three"], "a.f": True, "g": "10s"}


@pytest.mark.skipif(not os.path.exists(REF_CONF), reason="reference config not mounted")
def test_reference_application_conf_is_accepted():
    cfg = mc.Config().load_file(REF_CONF)
    assert cfg["mxar.remote.hostname"] == "127.0.0.1"
    assert cfg["mxar.remote.port"] == 0
    assert cfg.seeds() == ["akka.tcp://ClusterSystem@127.0.0.1:2551", "akka.tcp://ClusterSystem@127.0.0.1:2552"]
    assert cfg["mxar.cluster.auto-down-unreachable-after"] == 10.0
    assert cfg["mxar.loglevel"] == "INFO" and cfg["mxar.log-dead-letters"] == 5


def test_own_conf_and_layering():
    cfg = mc.Config().load_file(os.path.join(ROOT, "conf", "application.conf"))
    assert cfg["mxar.allreduce.th-reduce"] == 0.9 and cfg["mxar.allreduce.max-round"] == 100
    assert cfg["mxar.cluster.failure-detector.heartbeat-interval"] == 1.0
    cfg.load_env({"MXAR_ALLREDUCE_TH_REDUCE": "0.5", "MXAR_CLUSTER_SEED_NODES": "a,b", "UNRELATED": "1"})
    assert cfg["mxar.allreduce.th-reduce"] == 0.5 and cfg.seeds() == ["a", "b"]
    cfg.load_overrides(["mxar.allreduce.th-reduce=0.25", "akka.cluster.auto-down-unreachable-after=500ms"])
    assert cfg["mxar.allreduce.th-reduce"] == 0.25
    assert cfg["mxar.cluster.auto-down-unreachable-after"] == 0.5
    assert cfg.origin["mxar.allreduce.th-reduce"] == "cli"


def test_defaults_match_reference_constants():
    cfg = mc.Config()
    # AllreduceMaster.scala:105-114
    assert (cfg["mxar.allreduce.th-allreduce"], cfg["mxar.allreduce.th-reduce"], cfg["mxar.allreduce.th-complete"],
            cfg["mxar.allreduce.max-lag"], cfg["mxar.allreduce.max-round"]) == (1.0, 0.9, 0.8, 1, 100)
    assert cfg["mxar.allreduce.total-workers"] == 2 and cfg["mxar.allreduce.max-chunk-size"] == 2


def test_bad_input_errors():
    with pytest.raises(mc.ConfigError):
        mc.parse_hocon("a { b = 1")
    with pytest.raises(mc.ConfigError):
        mc.Config().load_overrides(["novalue"])
    with pytest.raises(mc.ConfigError):
        mc.as_seconds("ten seconds")

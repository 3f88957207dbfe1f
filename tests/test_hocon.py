"""HOCON (application.conf) configuration, the reference's config format."""
import os

import pytest

from sharetrade.config import Config
from sharetrade.utils import hocon

MAIN_CONF = """
# production profile: file journal, INFO logging
akka {
  loggers = ["akka.event.slf4j.Slf4jLogger"]
  loglevel = "INFO"
  persistence {
    journal {
      plugin = "akka.persistence.journal.leveldb"
      leveldb.dir = "var/journal"
      leveldb.compaction-intervals { some-actor = 1000, "*" = 5000 }
    }
    snapshot-store.plugin = "akka.persistence.snapshot-store.local"
    snapshot-store.local.dir = "var/snapshots"
  }
}
sharetrade.agent { lr = 0.005, optimizer = adam }
sharetrade.router.n_workers: 4
"""

TEST_CONF = """
akka {
// loggers = ["akka.event.slf4j.Slf4jLogger"]
  loglevel = "DEBUG"
  loggers = ["akka.testkit.TestEventListener"]
  persistence {
    journal.plugin = "inmemory-journal"
    snapshot-store.plugin = "inmemory-snapshot-store"
  }
}
"""


def test_parser_subset():
    t = hocon.loads('a { b.c = 1, d: "x y" }\na.b.e = [1, 2.5, true, null, "s"]\nf { g = off } # c\nh = plain')
    assert t == {"a": {"b": {"c": 1, "e": [1, 2.5, True, None, "s"]}, "d": "x y"}, "f": {"g": False},
                 "h": "plain"}
    assert hocon.get(t, "a.b.c") == 1 and hocon.get(t, "a.zz", 7) == 7
    with pytest.raises(hocon.HoconError):
        hocon.loads("a = ${b}")
    with pytest.raises(hocon.HoconError):
        hocon.loads("a { b = 1")


def test_akka_keys_map_to_config(tmp_path):
    p = tmp_path / "application.conf"
    p.write_text(MAIN_CONF)
    cfg = Config.load(str(p))
    assert cfg.persist.journal_plugin == "file" and cfg.persist.journal_dir == "var/journal"
    assert cfg.persist.snapshot_dir == "var/snapshots" and cfg.log.loglevel == "INFO"
    assert not cfg.log.test_listener
    assert cfg.agent.lr == 0.005 and cfg.agent.optimizer == "adam" and cfg.router.n_workers == 4
    _, ignored = hocon.akka_to_config(hocon.loads(MAIN_CONF))
    assert "akka.persistence.journal.leveldb.compaction-intervals" in ignored


def test_test_profile(tmp_path):
    p = tmp_path / "test.conf"
    p.write_text(TEST_CONF)
    cfg = Config.load(str(p))
    assert cfg.persist.journal_plugin == "inmemory" and cfg.log.loglevel == "DEBUG" and cfg.log.test_listener


@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="reference checkout not mounted")
def test_reference_conf_files_parse():
    for f in ("src/main/resources/application.conf", "src/test/resources/application.conf"):
        with open(os.path.join("/root/reference", f)) as fh:
            d, _ = hocon.akka_to_config(hocon.loads(fh.read()))
        assert d["persist"]["journal_plugin"] in ("file", "inmemory")

"""`.env` loading (reference app/main.py:23, app/rfq_agent.py:13): python-dotenv's
default semantics with the in-tree loader."""
import os
import subprocess
import sys

from replisense_rfq_amd.utils.dotenv import dotenv_values, find_dotenv, load_dotenv

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_parse_forms(tmp_path):
    p = tmp_path / ".env"
    p.write_text("# comment\nA=1\nexport B = two  # trailing\nC='lit ${A}'\n"
                 'D="x\\ny ${A}"\nE=${A}-${MISSING:-dflt}\n\nbad line\n')
    v = dotenv_values(p)
    assert v == {"A": "1", "B": "two", "C": "lit ${A}", "D": "x\ny 1", "E": "1-dflt"}


def test_no_override_and_find(tmp_path, monkeypatch):
    (tmp_path / "sub").mkdir()
    (tmp_path / ".env").write_text("RFQ_TEST_X=file\nRFQ_TEST_Y=file\n")
    monkeypatch.setenv("RFQ_TEST_X", "env")
    monkeypatch.delenv("RFQ_TEST_Y", raising=False)
    assert find_dotenv(start=tmp_path / "sub") == str(tmp_path / ".env")
    assert load_dotenv(find_dotenv(start=tmp_path / "sub"))
    assert os.environ["RFQ_TEST_X"] == "env" and os.environ["RFQ_TEST_Y"] == "file"
    monkeypatch.delenv("RFQ_TEST_Y")


def test_api_honours_dotenv(tmp_path):
    """MAX_FILE_SIZE_MB from a .env in the working directory reaches the API
    constants (read at import, after load_dotenv, as in the reference)."""
    (tmp_path / ".env").write_text("MAX_FILE_SIZE_MB=3\n")
    env = {k: v for k, v in os.environ.items() if k != "MAX_FILE_SIZE_MB"}
    env["PYTHONPATH"] = ROOT
    out = subprocess.run([sys.executable, "-c",
                          "from replisense_rfq_amd.api import main; print(main.MAX_FILE_SIZE_MB)"],
                         cwd=tmp_path, env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.strip().splitlines()[-1] == "3", out.stderr[-2000:]

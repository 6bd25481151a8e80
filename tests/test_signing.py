"""tools/sign.sh: detached GPG signatures of native sources."""

import os
import shutil
import subprocess

import pytest

from .helpers import ROOT


@pytest.mark.skipif(shutil.which("gpg") is None, reason="gpg not installed")
def test_sign_and_verify(tmp_path):
    home = tmp_path / "gnupg"
    home.mkdir(mode=0o700)
    env = dict(os.environ, GNUPGHOME=str(home))
    r = subprocess.run(["gpg", "--batch", "--passphrase", "", "--quick-gen-key", "mpx test <mpx@example.invalid>",
                        "ed25519", "sign", "never"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    src = tmp_path / "main.c"
    src.write_text("int main(void) { return 0; }\n")
    sign = os.path.join(ROOT, "tools", "sign.sh")
    r = subprocess.run([sign, str(src)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert (tmp_path / "main.c.asc").read_text().startswith("-----BEGIN PGP SIGNATURE-----")
    assert subprocess.run([sign, "--verify", str(src)], env=env, capture_output=True, timeout=120).returncode == 0
    src.write_text("int main(void) { return 1; }\n")  # tampered
    assert subprocess.run([sign, "--verify", str(src)], env=env, capture_output=True, timeout=120).returncode != 0

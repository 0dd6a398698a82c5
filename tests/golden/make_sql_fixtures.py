"""Regenerate tests/golden/sql/ from the reference checkout (run in the build container
only; the GPU box never reads /root/reference).

The fixtures are DATA: the reference's own parser test inputs (tests/sql/*.sql, checked
by tests/parser_test.rs:19-34 with `Parser::parse(sql).is_ok()`) and the two input
statements of its criterion bench (benches/parser_bench.rs:5,8-46).
"""
import re
import shutil
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "sql"


def main():
    OUT.mkdir(exist_ok=True)
    for f in sorted((REF / "tests" / "sql").glob("*.sql")):
        shutil.copyfile(f, OUT / f.name)
    src = (REF / "benches" / "parser_bench.rs").read_text()
    (OUT / "bench_short.sql").write_text(re.search(r'let short_sql = "([^"]*)";', src).group(1))
    (OUT / "bench_long.sql").write_text(re.search(r'let long_sql = r#"(.*?)"#;', src, re.S).group(1))


if __name__ == "__main__":
    main()

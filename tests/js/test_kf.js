// Unit tests of the shared frontend runtime (kubeflow_rm_amd/webapps/crud_backend/static/kf.js),
// the role of kubeflow-common-lib's Karma specs (poller.service.spec.ts, namespace.service.spec.ts):
// run by tests/test_frontend_js.py with the system node, no browser.
"use strict";
const assert = require("assert");
const path = require("path");

// minimal browser globals kf.js touches at load time
const listeners = {};
const posted = [];
global.window = global;
global.document = { cookie: "XSRF-TOKEN=tok%3D1; other=2" };
global.location = { search: "" };
const store = {};
global.localStorage = { getItem: (k) => store[k] || null, setItem: (k, v) => { store[k] = String(v); } };
global.addEventListener = (t, f) => { listeners[t] = f; };
global.parent = { postMessage: (m) => posted.push(m) };  // inside the dashboard iframe
const timers = [];
global.setTimeout = (f, ms) => { timers.push(ms); return timers.length; };
global.clearTimeout = () => {};

const kf = require(path.join(__dirname, "../../kubeflow_rm_amd/webapps/crud_backend/static/kf.js"));
const tests = [];
const test = (name, fn) => tests.push([name, fn]);

test("iframe announces itself to the dashboard (library.js protocol)", () => {
  assert.deepStrictEqual(posted[0], { type: "iframe-connected" });
});

test("namespace-selected from the parent drives the namespace service", () => {
  const seen = [];
  kf.onNamespace((ns) => seen.push(ns));
  listeners.message({ data: { type: "namespace-selected", value: "team-a" } });
  listeners.message({ data: { type: "namespace-selected", value: "team-a" } });  // no duplicate
  assert.deepStrictEqual(seen, ["team-a"]);
  assert.strictEqual(kf.namespace(), "team-a");
  assert.strictEqual(store["kf-namespace"], "team-a");
  listeners.message({ data: { type: "parent-connected" } });
  assert.deepStrictEqual(posted[posted.length - 1], { type: "iframe-connected" });
});

test("cookie reader (CSRF double submit)", () => {
  assert.strictEqual(kf.cookie("XSRF-TOKEN"), "tok=1");
  assert.strictEqual(kf.cookie("missing"), "");
});

test("poller backs off 1 -> 2 -> 4 -> 8 s while unchanged and resets on change", async () => {
  timers.length = 0;
  let value = 1;
  const p = new kf.Poller(async () => value);
  await p.tick();   // first data: changed -> min
  await p.tick();   // unchanged
  await p.tick();
  await p.tick();
  await p.tick();   // capped
  value = 2;
  await p.tick();   // changed -> reset
  assert.deepStrictEqual(timers, [1000, 2000, 4000, 8000, 8000, 1000]);
});

test("toYaml renders API objects in block style", () => {
  const y = kf.toYaml({ apiVersion: "v1", kind: "PersistentVolumeClaim",
    metadata: { name: "ws", labels: {}, annotations: { "a/b": "true" } },
    spec: { accessModes: ["ReadWriteOnce"], resources: { requests: { storage: "5Gi" } } },
    status: { conditions: [{ type: "Ready", status: "True" }], count: 3, empty: [] } });
  assert.strictEqual(y, [
    "apiVersion: v1", "kind: PersistentVolumeClaim", "metadata:", "  name: ws", "  labels: {}",
    "  annotations:", '    a/b: "true"', "spec:", "  accessModes:", "  - ReadWriteOnce", "  resources:",
    "    requests:", "      storage: 5Gi", "status:", "  conditions:", "  - type: Ready", '    status: "True"',
    "  count: 3", "  empty: []"].join("\n"));
});

test("escaping of API strings before they reach innerHTML", () => {
  assert.strictEqual(kf.esc('<img src=x onerror="a">'), "&lt;img src=x onerror=&quot;a&quot;&gt;");
  assert.ok(kf.statusCell({ phase: "warning", message: '"><script>' }).indexOf("<script>") < 0);
});

test("events table sorts newest first", () => {
  const html = kf.eventsTable([{ type: "Normal", reason: "Old", lastTimestamp: "2024-01-01T00:00:00Z" },
                               { type: "Warning", reason: "New", lastTimestamp: "2024-01-02T00:00:00Z" }]);
  assert.ok(html.indexOf("New") < html.indexOf("Old"));
  assert.ok(kf.eventsTable([]).includes("No events"));
});

test("parseYaml: the block YAML the apps exchange (js-yaml load semantics)", () => {
  const [v, err] = kf.parseYaml([
    "apiVersion: v1",
    "kind: PersistentVolumeClaim   # trailing comment",
    "metadata:",
    '  name: "{notebook-name}-data"',
    "  labels: {app: x, n: 3, 'q': [a, \"b\"]}",
    "spec:",
    "  accessModes:",
    "  - ReadWriteOnce",       // sequence at its key's indent
    "  resources:",
    "    requests:",
    "      storage: 20Gi",
    "  items:",
    "    - name: a",          // compact mapping items
    "      value: 1.5",
    "    -",
    "      - nested",
    "  script: |",
    "    echo hi",
    "",
    "    exit 0",
    "  folded: >-",
    "    a b",
    "    c",
    "  empty:",
    "  quoted: 'it''s # not a comment'",
    "  flags: [true, false, null, ~, 0x1f, -3, .inf]",
    "---",
  ].join("\n"));
  assert.strictEqual(err, "");
  assert.deepStrictEqual(v, {
    apiVersion: "v1", kind: "PersistentVolumeClaim",
    metadata: { name: "{notebook-name}-data", labels: { app: "x", n: 3, q: ["a", "b"] } },
    spec: { accessModes: ["ReadWriteOnce"], resources: { requests: { storage: "20Gi" } },
            items: [{ name: "a", value: 1.5 }, ["nested"]], script: "echo hi\n\nexit 0\n", folded: "a b c",
            empty: null, quoted: "it's # not a comment", flags: [true, false, null, null, 31, -3, Infinity] },
  });
  assert.deepStrictEqual(kf.parseYaml(""), [{}, ""]);
  assert.deepStrictEqual(kf.parseYaml("- a\n- b: 1\n  c: 2"), [["a", { b: 1, c: 2 }], ""]);
});

test("parseYaml: errors carry the reason and line:column, value {} (parseYAML contract)", () => {
  assert.deepStrictEqual(kf.parseYaml("a: 1\n  b: 2"), [{}, "bad indentation of a mapping entry (2:3)"]);
  assert.deepStrictEqual(kf.parseYaml("a: 1\na: 2"), [{}, "duplicated mapping key (2:1)"]);
  assert.deepStrictEqual(kf.parseYaml("a:\n\t- x"), [{}, "tab characters must not be used in indentation (2:1)"]);
  assert.ok(kf.parseYaml("a: [1, 2").at === undefined && kf.parseYaml("a: [1, 2")[1].startsWith("missed comma"));
  assert.ok(kf.parseYaml('a: "x\\q').at === undefined && kf.parseYaml('a: "x')[1].startsWith("bad double-quoted scalar"));
  assert.ok(kf.parseYaml("a: 1\n- b")[1].startsWith("bad indentation of a sequence entry"));
});

test("toYaml -> parseYaml round-trips API objects (quoting of numeric / boolean strings)", () => {
  const o = { metadata: { name: "nb", annotations: { "notebooks.kubeflow.org/last-activity": "2024-01-01T00:00:00Z", b: "true", n: "1.0", e: "" } },
              spec: { template: { spec: { containers: [{ name: "c", args: ["--port", "8888"], env: [], resources: { limits: { "amd.com/gpu": 2 } } }] } } },
              status: { conditions: [], readyReplicas: 1, msg: "two\nlines", colon: "a: b", hash: "x #y" } };
  assert.deepStrictEqual(kf.parseYaml(kf.toYaml(o)), [o, ""]);
});

test("highlightYaml: keys, strings, numbers, comments and dashes as token spans", () => {
  const h = kf.highlightYaml('a: "x" # c\n- 3\nb: <tag>');
  assert.ok(h.includes('<span class="y-k">a</span>: <span class="y-s">&quot;x&quot;</span> <span class="y-c"># c</span>'), h);
  assert.ok(h.includes('<span class="y-p">-</span> <span class="y-n">3</span>'), h);
  assert.ok(h.includes('<span class="y-v">&lt;tag&gt;</span>'), h);  // escaped
});

(async () => {
  let failed = 0;
  for (const [name, fn] of tests) {
    try { await fn(); console.log(`ok - ${name}`); } catch (e) { failed++; console.log(`not ok - ${name}\n${e.stack}`); }
  }
  console.log(`${tests.length - failed}/${tests.length} passed`);
  process.exit(failed ? 1 : 0);
})();

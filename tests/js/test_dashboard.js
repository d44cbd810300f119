// Central dashboard contract tests (node, no browser): cdb.js against the reference's specs.
//   centraldashboard-angular/frontend/cypress/e2e/namespace-selector.cy.ts  (+ fixtures/envinfo.json)
//   centraldashboard-angular/frontend/cypress/e2e/url-syncing.cy.ts         (browser <-> iframe URLs)
//   centraldashboard/public/components/main-page_test.js      (menu hrefs, active item, iframe src)
//   centraldashboard/public/components/activities-list_test.js, registration-page_test.js
// argv[2] = /root/reference/components (fixtures are read in place).
"use strict";
const assert = require("assert");
const fs = require("fs");
const path = require("path");

const C = require(path.join(__dirname, "../../kubeflow_rm_amd/webapps/dashboard/static/cdb.js"));
const REF = process.argv[2];
const fixture = (name) => JSON.parse(fs.readFileSync(
  path.join(REF, "centraldashboard-angular/frontend/cypress/fixtures", name + ".json"), "utf8"));

const tests = [];
const test = (name, fn) => tests.push([name, fn]);

// One page load: the selector's visible text for a browser URL and a stored choice.
function selected(envInfo, url, stored) {
  const opts = C.namespaceOptions(envInfo.namespaces, url);
  const q = C.queryParams(url.split("?")[1] ? "?" + url.split("?")[1].split("#")[0] : "");
  const ns = C.pickNamespace(opts, { queryNs: q.ns, storedNs: stored });
  const html = C.renderNamespaceSelector(opts, ns);
  const m = html.match(/data-cy-selected-namespace>([\s\S]*?)<\/button>/);
  return { text: m[1].replace(/<[^>]+>/g, ""), ns, html };
}

// ---- namespace-selector.cy.ts ------------------------------------------------------------------
test("namespace from the query parameters (every fixture namespace)", () => {
  const env = fixture("envinfo");
  for (const n of env.namespaces) assert.ok(selected(env, `/?ns=${n.namespace}`, "test-namespace-2").text.includes(n.namespace));
});

test("an invalid ?ns= is not selected", () => {
  assert.ok(!selected(fixture("envinfo"), "/?ns=invalid-namespace", "test-namespace-2").text.includes("invalid-namespace"));
});

test("All namespaces is not selectable on the home page", () => {
  assert.ok(!selected(fixture("envinfo"), "/?ns=All namespaces", "test-namespace-2").text.includes("All namespaces"));
});

test("All namespaces in the allowed apps, and not after going Home", () => {
  const env = fixture("envinfo");
  assert.ok(selected(env, "/_/jupyter?ns=All namespaces", "test-namespace-2").text.includes("All namespaces"));
  assert.ok(selected(env, "/_/volumes?ns=All namespaces", "test-namespace-2").text.includes("All namespaces"));
  // the Home menu item keeps ?ns=All namespaces, which is not valid there
  const home = C.renderSidenav([], "All namespaces", "/_/jupyter?ns=All namespaces", {});
  const href = home.match(/href="([^"]+)"[^>]*data-cy-sidenav-menu-item="Home"/)[1].replace(/&amp;/g, "&");
  assert.ok(!selected(env, decodeURIComponent(href.replace(/\+/g, " ")), "All namespaces").text.includes("All namespaces"));
  // and not in an app outside the list
  assert.ok(!selected(env, "/_/pipeline/?ns=All namespaces", "x").text.includes("All namespaces"));
});

test("namespace from local storage; an invalid stored one is ignored", () => {
  const env = fixture("envinfo");
  assert.ok(selected(env, "/", "test-namespace-2").text.includes("test-namespace-2"));
  assert.ok(!selected(env, "/", "invalid-namespace").text.includes("invalid-namespace"));
  assert.strictEqual(C.storageKey("user"), "selectedNamespace/.user");
});

test("otherwise the namespace with the Owner role, then the first namespace", () => {
  const env = fixture("envinfo");
  assert.ok(selected(env, "/", null).text.includes("kubeflow-user"));
  const env2 = JSON.parse(JSON.stringify(env));
  env2.namespaces[1].role = "";
  assert.ok(selected(env2, "/", null).text.includes("test-namespace-1"));
});

test("No namespaces", () => {
  const env = fixture("envinfo");
  env.namespaces = [];
  const r = selected(env, "/", null);
  assert.ok(r.text.includes("No namespaces"));
  assert.ok(r.html.includes('class="ns-trigger disabled"'));
});

test("(Owner) shown for an owned selection and in the option list", () => {
  const env = fixture("envinfo");
  const r = selected(env, "/?ns=kubeflow-user", null);
  assert.ok(r.text.includes("(Owner)"));
  assert.ok(r.html.includes('data-cy-namespace="kubeflow-user"'));
  assert.ok(!selected(env, "/?ns=test-namespace-1", null).text.includes("(Owner)"));
});

// ---- url-syncing.cy.ts -------------------------------------------------------------------------
function harness(origin) {
  const frameLoc = { href: "about:blank", pathname: "", search: "", hash: "" };
  const history = [];
  let browser = "/";
  const router = {
    url: () => browser,
    navigate(p, params, frag) {
      browser = p + C.queryString(params) + (frag !== undefined ? "#" + frag : "");
      history.push(browser);
    },
  };
  const sync = new C.IframeSync(router, () => ({ location: frameLoc }), () => "kubeflow-user");
  const load = (src) => {  // the iframe loads src (origin-absolute or path)
    const u = new URL(src, origin);
    Object.assign(frameLoc, { href: u.href, pathname: u.pathname, search: u.search, hash: u.hash });
  };
  const equalUrls = () => C.sameUrl(C.stripPrefix(browser), frameLoc.pathname + frameLoc.search + frameLoc.hash);
  return { sync, load, frameLoc, history, get browser() { return browser; }, set browser(v) { browser = v; }, equalUrls };
}

test("menu click loads the app; navigating inside the app mirrors the browser URL", () => {
  const O = "https://kf.example";
  const h = harness(O);
  const links = fixture("dashboardlinks").menuLinks;
  const nb = links.find((l) => l.text === "Notebooks");
  h.browser = C.menuHref(nb.link, "kubeflow-user");
  const src = h.sync.onNavigate(h.browser, O, true);
  assert.strictEqual(src, O + "/jupyter/?ns=kubeflow-user");
  h.load(src);
  h.sync.tick();
  assert.ok(h.equalUrls());
  // New Notebook button inside the app
  h.load(O + "/jupyter/new");
  assert.ok(h.sync.tick());
  assert.strictEqual(h.browser, "/_/jupyter/new?ns=kubeflow-user");
  assert.ok(h.equalUrls());
  // the browser route change caused by the mirroring must not reload the iframe
  assert.strictEqual(h.sync.onNavigate(h.browser, O, false), null);
  // back arrow inside the app
  h.load(O + "/jupyter/");
  h.sync.tick();
  assert.ok(h.equalUrls());
  // the notebook details page (query parameters + fragment carried over)
  h.load(O + "/jupyter/notebook/details/kubeflow-user/test-notebook?tab=logs#top");
  h.sync.tick();
  assert.strictEqual(h.browser, "/_/jupyter/notebook/details/kubeflow-user/test-notebook?tab=logs&ns=kubeflow-user#top");
  assert.ok(h.equalUrls());
  assert.ok(h.history.length >= 3);  // one history entry per app page
});

test("cross-app link (JWA -> VWA details) and back through the sidebar", () => {
  const O = "https://kf.example";
  const h = harness(O);
  h.load(h.sync.onNavigate("/_/jupyter/?ns=kubeflow-user", O, true));
  h.sync.tick();
  h.load(O + "/volumes/details/kubeflow-user/test-notebook-volume");
  h.sync.tick();
  assert.strictEqual(h.browser, "/_/volumes/details/kubeflow-user/test-notebook-volume?ns=kubeflow-user");
  assert.ok(h.equalUrls());
  // sidebar link back to the app index: forced reload even though the app is the same one
  const src = h.sync.onNavigate("/_/jupyter/?ns=kubeflow-user", O, true);
  assert.ok(src !== null && src.endsWith("/jupyter/?ns=kubeflow-user"));
  const again = h.sync.onNavigate("/_/jupyter/?ns=kubeflow-user", O, true);
  assert.notStrictEqual(again, src);  // the value alternates so the iframe reloads
});

test("a query-parameter change inside the app keeps the namespace in the browser URL", () => {
  const O = "https://kf.example";
  const h = harness(O);
  h.load(O + "/jupyter/?sort=name");
  h.sync.tick();
  assert.deepStrictEqual(C.queryParams(h.browser.split("?")[1]), { sort: "name", ns: "kubeflow-user" });
  // an ns carried by the app itself wins
  h.load(O + "/volumes/?ns=other");
  h.sync.tick();
  assert.strictEqual(C.queryParams(h.browser.split("?")[1]).ns, "other");
  // URLs that differ only in ns / a trailing slash are the same page
  assert.ok(C.sameUrl("/jupyter?ns=a", "/jupyter/?ns=b"));
  assert.ok(!C.sameUrl("/jupyter/?x=1", "/jupyter/?x=2"));
  assert.ok(!C.sameUrl("/jupyter/#a", "/jupyter/#b"));
});

// ---- main-page_test.js (Polymer dashboard) -----------------------------------------------------
const MENU_LINKS = [
  { link: "/jupyter/", text: "Notebooks" },
  { link: "/pipeline/#/pipelines", text: "Pipelines" },
  { link: "/katib/trials", text: "Katib Trials" },
  { type: "section", text: "Experiments", items: [
    { link: "/pipeline/#/experiments", text: "Pipelines" },
    { link: "/katib/experiments", text: "Katib Experiments" }] },
  { link: "/pipeline/#/runs", text: "Runs" },
  { link: "/myapp/{ns}", text: "MyApp" },
];

test("links carry ?ns= only when a namespace is selected", () => {
  const none = C.renderSidenav(MENU_LINKS, "", "/", {});
  for (const m of none.matchAll(/href="([^"]+)"/g)) assert.ok(!m[1].includes("?"), m[1]);
  const some = C.renderSidenav(MENU_LINKS, "another-namespace", "/", {});
  for (const m of some.matchAll(/href="([^"]+)"/g)) assert.ok(m[1].includes("?ns=another-namespace"), m[1]);
});

test("active menu item: simple, hash-based and path-based common prefixes, namespaced", () => {
  assert.strictEqual(C.activeMenuLink(MENU_LINKS, "/_/jupyter/").link, "/jupyter/");
  assert.strictEqual(C.activeMenuLink(MENU_LINKS, "/_/pipeline/#/experiments/details/12345").link, "/pipeline/#/experiments");
  assert.strictEqual(C.activeMenuLink(MENU_LINKS, "/_/pipeline/#/runs/details/12345").link, "/pipeline/#/runs");
  assert.strictEqual(C.activeMenuLink(MENU_LINKS, "/_/katib/experiments/id/12345").link, "/katib/experiments");
  assert.strictEqual(C.activeMenuLink(MENU_LINKS, "/_/katib/trials/id/12345").link, "/katib/trials");
  assert.strictEqual(C.activeMenuLink(MENU_LINKS, "/_/myapp/test", "test").link, "/myapp/{ns}");
  assert.strictEqual(C.menuHref("/myapp/{ns}", "test"), "/_/myapp/test?ns=test");
  const html = C.renderSidenav(MENU_LINKS, "test", "/_/katib/trials/id/1", {});
  assert.strictEqual((html.match(/class="active"/g) || []).length, 1);
  assert.ok(/class="active" data-cy-sidenav-menu-item="Katib Trials"/.test(html));
});

test("views: iframe src keeps query + hash; unresolved {ns} -> namespace-needed; unknown -> 404", () => {
  assert.deepStrictEqual(C.viewFor("/_/pipeline/?ns=test&foo=bar#/hash/route/fragments"),
                         { page: "iframe", src: "/pipeline/?ns=test&foo=bar#/hash/route/fragments" });
  assert.strictEqual(C.viewFor("/").page, "home");
  assert.strictEqual(C.viewFor("/manage-users").page, "manage-users");
  assert.deepStrictEqual(C.viewFor("/_/myapp/{ns}"), { page: "namespace-needed", path: "/_/myapp/{ns}" });
  assert.deepStrictEqual(C.viewFor("/_/myapp/%7Bns%7D"), { page: "namespace-needed", path: "/_/myapp/{ns}" });
  assert.deepStrictEqual(C.viewFor("/not/a/page"), { page: "not-found", path: "/not/a/page" });
  assert.ok(C.renderNotFound("/not/<b>").includes("Sorry, <b>/not/&lt;b&gt;</b> is not a valid page."));
  assert.ok(C.renderNamespaceNeeded().includes("requires a namespace"));
  // a menu link with {ns} and no namespace stays unresolved -> namespace-needed
  assert.strictEqual(C.viewFor(C.menuHref("/myapp/{ns}", "")).page, "namespace-needed");
});

test("build label / version / id in the sidenav footer", () => {
  const env = fixture("envinfo");
  const html = C.renderSidenav([], "", "/", env.platform);
  assert.ok(html.includes('<span class="buildVersion">Build Label Version</span>'));
  assert.ok(html.includes('<span class="buildId">Build Label Id</span>'));
});

// ---- activities-list_test.js -------------------------------------------------------------------
test("activities grouped by day, newest first, errors flagged", () => {
  const now = new Date(2026, 9, 16, 21, 0, 0);
  const yesterday = new Date(now - 86400000);
  const html = C.renderActivities([
    { lastTimestamp: yesterday.toISOString(), message: "Something bad happened", type: "Warning", involvedObject: { name: "a-failing-pod" } },
    { lastTimestamp: now.toISOString(), message: "Something happened", type: "Normal", involvedObject: { name: "some-pod" } }], now);
  assert.strictEqual((html.match(/class="activity-row"/g) || []).length, 2);
  assert.deepStrictEqual([...html.matchAll(/<h2>([^<]*)<\/h2>/g)].map((m) => m[1]), ["Today", "Yesterday"]);
  assert.strictEqual((html.match(/class="icon error"/g) || []).length, 1);
  const base = new Date(2026, 9, 16, 20, 0, 0);
  const evs = [], want = [];
  for (let i = 10; i > 0; i--) {
    const d = new Date(base - i * 3600000);
    evs.push({ lastTimestamp: d.toISOString(), message: `m${i}`, type: "Normal", involvedObject: { name: "p" } });
    want.push(d.toLocaleTimeString());
  }
  const h2 = C.renderActivities(evs, base);
  assert.deepStrictEqual([...h2.matchAll(/<span class="time">([^<]*)<\/span>/g)].map((m) => m[1]), want.reverse());
  assert.ok(C.renderActivities([], now).includes("No activities"));
});

// ---- registration-page_test.js -----------------------------------------------------------------
test("registration: name rule, create + poll until the workgroup exists, error surfaced", async () => {
  assert.strictEqual(C.validateNamespace("kubeflow-"), C.NS_RULE_MESSAGE);
  assert.strictEqual(C.validateNamespace("kubeflow-user"), null);
  assert.strictEqual(C.suggestNamespace("Jane.Doe_1@example.com"), "jane-doe1");
  let created = null, polls = 0;
  const api = { create: async (ns) => { created = ns; }, exists: async () => ({ hasWorkgroup: ++polls >= 3 }) };
  const ok = await C.register(api, "kubeflow-user", { sleep: async () => {} });
  assert.deepStrictEqual(ok, { ok: true });
  assert.strictEqual(created, "kubeflow-user");
  assert.strictEqual(polls, 3);
  // API DB never consistent within the poll budget
  const slow = await C.register({ create: async () => {}, exists: async () => ({ hasWorkgroup: false }) }, "x", { times: 5, sleep: async () => {} });
  assert.strictEqual(slow.ok, false);
  // server-side error shown, no polling
  let p2 = 0;
  const bad = await C.register({ create: async () => { throw new Error("Test Error!"); }, exists: async () => { p2++; return {}; } }, "ns");
  assert.deepStrictEqual(bad, { ok: false, error: "Test Error!" });
  assert.strictEqual(p2, 0);
  // client-side validation stops before the API
  let called = false;
  const inval = await C.register({ create: async () => { called = true; }, exists: async () => ({}) }, "kubeflow-");
  assert.strictEqual(inval.error, C.NS_RULE_MESSAGE);
  assert.strictEqual(called, false);
});

test("recent notebooks: five most recent, escaped contributors table", () => {
  const rows = Array.from({ length: 8 }, (_, i) => ({ name: `nb-${i}`, age: new Date(2026, 0, 1 + i).toISOString() }));
  assert.deepStrictEqual(C.recentNotebooks(rows).map((r) => r.name), ["nb-7", "nb-6", "nb-5", "nb-4", "nb-3"]);
  const t = C.renderContributors("ns", ["a@x.io", "<script>"]);
  assert.ok(t.includes("&lt;script&gt;") && !t.includes("<script>"));
});

(async () => {
  let failed = 0;
  for (const [name, fn] of tests) {
    try {
      await fn();
      console.log("ok  ", name);
    } catch (e) {
      failed++;
      console.log("FAIL", name, "\n", e && e.stack);
    }
  }
  console.log(`${tests.length - failed}/${tests.length} passed`);
  process.exit(failed ? 1 : 0);
})();
